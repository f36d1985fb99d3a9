set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x -k "gemm or linear or fused_output" --timeout 120 --timeout-method thread > gpurun_out/s3_split_tests.log 2>&1
timeout -k 10 120 python scripts/gemm_kscale.py > gpurun_out/s3_split_kscale.log 2>&1
timeout -k 10 200 python bench.py > gpurun_out/s3_split_bench.log 2>&1
