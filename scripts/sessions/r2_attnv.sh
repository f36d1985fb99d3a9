set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
o=gpurun_out/r2attnv.txt
: > $o
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_gpu_e2e.py -k "attention or attn or e2e" > gpurun_out/r2attnv_tests.log 2>&1
for i in 1 2; do
for lib in old new; do
  if [ $lib = old ]; then export LJS_KERNELS_LIB=$PWD/learning_jax_sharding_amd/_lib/libljs_kernels_old.so; else unset LJS_KERNELS_LIB; fi
  echo "$lib $(timeout -k 10 120 python scripts/attn_time.py 2>&1 | tail -1)" >> $o
  echo "$lib b64 $(timeout -k 10 200 python bench.py --steps 200 --warmup 20 2>&1 | grep -o '"ms_per_step": [0-9.]*')" >> $o
done
done
