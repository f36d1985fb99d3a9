set -e
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k "fp8" > gpurun_out/r2f8_tests.log 2>&1
timeout -k 10 300 python scripts/fp8_bench.py > gpurun_out/r2f8_bench.log 2>&1
