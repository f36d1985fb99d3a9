set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
o=gpurun_out/r2adamab.txt
: > $o
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_epilogue_gpu.py tests/test_kernels_gpu.py -k "deferred or adam" > gpurun_out/r2adamab_tests.log 2>&1
for i in 1 2; do
for lib in old new; do
  if [ $lib = old ]; then export LJS_KERNELS_LIB=$PWD/learning_jax_sharding_amd/_lib/libljs_kernels_old.so; else unset LJS_KERNELS_LIB; fi
  echo "$lib b64 $(timeout -k 10 200 python bench.py --steps 200 --warmup 20 2>&1 | grep -o '"ms_per_step": [0-9.]*')" >> $o
  echo "$lib b8 $(timeout -k 10 200 python bench.py --steps 200 --warmup 20 --batch-per-gpu 8 2>&1 | grep -o '"ms_per_step": [0-9.]*')" >> $o
done
done
unset LJS_KERNELS_LIB
for m in "--model layer" "--model layer --fp8" "--model ff" "--model ff --fp8"; do
  echo "$m $(timeout -k 10 200 python bench.py --steps 100 --warmup 20 $m 2>&1 | grep -o '"ms_per_step": [0-9.]*')" >> $o
  echo "$m nodefer $(LJS_DEFER_WGRAD=0 timeout -k 10 200 python bench.py --steps 100 --warmup 20 $m 2>&1 | grep -o '"ms_per_step": [0-9.]*')" >> $o
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r2adamab_b64 -o prof -- python bench.py --steps 20 --warmup 5 > gpurun_out/r2adamab_b64.log 2>&1
