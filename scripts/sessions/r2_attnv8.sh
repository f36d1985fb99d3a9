set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
o=gpurun_out/r2attnv8.txt
: > $o
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_gpu_e2e.py -k "attention or attn or e2e or ring" > gpurun_out/r2attnv8_tests.log 2>&1
for i in 1 2; do
for lib in old new; do
  if [ $lib = old ]; then export LJS_KERNELS_LIB=$PWD/learning_jax_sharding_amd/_lib/libljs_kernels_old.so; else unset LJS_KERNELS_LIB; fi
  echo "$lib $(timeout -k 10 120 python scripts/attn_time.py 8 256 8 2>&1 | tail -1)" >> $o
  echo "$lib b8 $(timeout -k 10 200 python bench.py --steps 200 --warmup 20 --batch-per-gpu 8 2>&1 | grep -o '"ms_per_step": [0-9.]*')" >> $o
done
done
