set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
AB=learning_jax_sharding_amd/_lib/libljs_kernels_ab.so
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k "gemm or slab or weight_grad or linear" > gpurun_out/r2p_tests.log 2>&1
o=gpurun_out/r2p_ab.txt
: > $o
for cfg in "qkv 2561 1" "qkv 1282 1" "out 1602 1" "dwslab:640:1536 1282 8" "dwslab:2560:640 1282 5" "dwslab:512:640 1282 24"; do
  echo "new $(timeout -k 10 120 python scripts/gemm_one.py $cfg 50 2>&1 | grep -v amdgpu.ids)" >> $o
  echo "old $(LJS_KERNELS_LIB=$PWD/$AB timeout -k 10 120 python scripts/gemm_one.py $cfg 50 2>&1 | grep -v amdgpu.ids)" >> $o
done
for m in "" "--model layer" "--batch-per-gpu 8"; do
  echo "new $m $(timeout -k 10 200 python bench.py --steps 100 --warmup 20 $m 2>&1 | grep -o '"ms_per_step": [0-9.]*')" >> $o
  echo "old $m $(LJS_KERNELS_LIB=$PWD/$AB timeout -k 10 200 python bench.py --steps 100 --warmup 20 $m 2>&1 | grep -o '"ms_per_step": [0-9.]*')" >> $o
done
