set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_gpu_e2e.py -q -x -k "gemm or linear or sum or e2e or train" --timeout 120 --timeout-method thread > gpurun_out/s3_psum_tests.log 2>&1
timeout -k 10 200 python bench.py > gpurun_out/s3_psum_bench.log 2>&1
LJS_FUSED_SUM=0 timeout -k 10 200 python bench.py >> gpurun_out/s3_psum_bench.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof12 -o run -- python bench.py --steps 25 --warmup 5 > gpurun_out/prof12.log 2>&1
