set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_gpu_e2e.py tests/test_epilogue_gpu.py -x -q --timeout 200 --timeout-method thread -k "weight_grad or linear or slab or e2e or layer or attention_block" > gpurun_out/r2dws2_tests.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r2dws2_b8 -o prof -- python bench.py --steps 20 --warmup 5 --batch-per-gpu 8 > gpurun_out/r2dws2_b8.log 2>&1
