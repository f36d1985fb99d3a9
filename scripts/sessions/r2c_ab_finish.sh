set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/r2c_ab_finish.log
OLD=$GRAFT_REPO_ROOT/learning_jax_sharding_amd/_lib/libljs_kernels_old.so
for rep in 1 2 3; do
  for lib in old new; do
    for a in "--seq 4096 --batch-per-gpu 4" "--batch-per-gpu 8" ""; do
      if [ $lib = old ]; then r=$(LJS_KERNELS_LIB=$OLD timeout -k 10 120 python bench.py --steps 48 --warmup 8 $a | tail -1 | python -c "import json,sys; print(json.loads(sys.stdin.read())['ms_per_step'])");
      else r=$(timeout -k 10 120 python bench.py --steps 48 --warmup 8 $a | tail -1 | python -c "import json,sys; print(json.loads(sys.stdin.read())['ms_per_step'])"); fi
      echo "$lib [$a] $r" >> $out
    done
  done
done
