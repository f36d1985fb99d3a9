set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_gpu_e2e.py -q -x -k "attention or attn or ring or softmax" --timeout 120 --timeout-method thread > gpurun_out/r2c_resc2_tests.log 2>&1
out=gpurun_out/r2c_ab_resc2.log
OLD=$GRAFT_REPO_ROOT/learning_jax_sharding_amd/_lib/libljs_kernels_old.so
for rep in 1 2; do
  for lib in old new; do
    for a in "--seq 4096 --batch-per-gpu 4 --mode fwd" "--seq 4096 --batch-per-gpu 4" ""; do
      if [ $lib = old ]; then r=$(LJS_KERNELS_LIB=$OLD timeout -k 10 120 python bench.py --steps 48 --warmup 8 $a | tail -1 | python -c "import json,sys; print(json.loads(sys.stdin.read())['ms_per_step'])");
      else r=$(timeout -k 10 120 python bench.py --steps 48 --warmup 8 $a | tail -1 | python -c "import json,sys; print(json.loads(sys.stdin.read())['ms_per_step'])"); fi
      echo "$lib [$a] $r" >> $out
    done
  done
done
