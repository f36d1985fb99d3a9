set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
o=gpurun_out/r2const.txt
: > $o
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_epilogue_gpu.py tests/test_gpu_e2e.py tests/test_distributed_gpu.py -k "linear or dense or bias or e2e or jit or layer or slab or dp" > gpurun_out/r2const_tests.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r2const_b64 -o prof -- python bench.py --steps 20 --warmup 5 > gpurun_out/r2const_b64.log 2>&1
for i in 1 2; do
  echo "b64 $(timeout -k 10 200 python bench.py --steps 200 --warmup 20 2>&1 | grep -o '"ms_per_step": [0-9.]*')" >> $o
  echo "b8 $(timeout -k 10 200 python bench.py --steps 200 --warmup 20 --batch-per-gpu 8 2>&1 | grep -o '"ms_per_step": [0-9.]*')" >> $o
done
