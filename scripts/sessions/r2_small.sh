set -e
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python scripts/gemm_small.py > gpurun_out/r2s_small.log 2>&1
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k "gemm" > gpurun_out/r2s_tests.log 2>&1
