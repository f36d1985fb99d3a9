set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_gpu_e2e.py -q -x -k "adam or attention or e2e or train" --timeout 120 --timeout-method thread > gpurun_out/s3_adam_tests.log 2>&1
timeout -k 10 100 python scripts/small_kernels.py adam > gpurun_out/s3_adam_small.log 2>&1
timeout -k 10 200 python bench.py > gpurun_out/s3_adam_b64.log 2>&1
timeout -k 10 200 python bench.py --batch-per-gpu 8 > gpurun_out/s3_adam_b8.log 2>&1
