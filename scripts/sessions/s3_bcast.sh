set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_gpu_e2e.py -q -x -k "linear or sum or e2e or train or broadcast" --timeout 120 --timeout-method thread > gpurun_out/s3_bcast_tests.log 2>&1
timeout -k 10 200 python bench.py > gpurun_out/s3_bcast_bench.log 2>&1
