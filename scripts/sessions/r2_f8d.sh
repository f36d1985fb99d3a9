set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py tests/test_epilogue_gpu.py -x -q --timeout 200 --timeout-method thread -k "gemm or slab or weight_grad or linear or fp8 or epilogue or ff_block or layer or adam" > gpurun_out/r2e2_tests.log 2>&1
timeout -k 10 200 python bench.py --steps 50 --warmup 10 --model layer > gpurun_out/r2e2_layer_bf16.log 2>&1
timeout -k 10 200 python bench.py --steps 50 --warmup 10 --model layer --fp8 > gpurun_out/r2e2_layer_fp8.log 2>&1
timeout -k 10 200 python bench.py --steps 50 --warmup 10 > gpurun_out/r2e2_b64.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r2e2_prof -o prof -- python bench.py --steps 20 --warmup 5 --model layer --fp8 > gpurun_out/r2e2_prof.log 2>&1
