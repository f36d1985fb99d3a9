set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_gpu_e2e.py -q -x -k "ticket or sum or adam or e2e or train" --timeout 120 --timeout-method thread > gpurun_out/s3_tick_tests.log 2>&1
timeout -k 10 100 python scripts/small_kernels.py > gpurun_out/s3_tick_small.log 2>&1
timeout -k 10 200 python bench.py > gpurun_out/s3_tick_step.log 2>&1
