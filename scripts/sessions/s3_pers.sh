set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x -k "gemm or linear" --timeout 120 --timeout-method thread > gpurun_out/s3_pers_tests.log 2>&1
timeout -k 10 120 python scripts/gemm_kscale.py > gpurun_out/s3_pers_kscale.log 2>&1
for t in 0 1; do LJS_GEMM_TILE2561=$t timeout -k 10 200 python bench.py | sed "s/^/t2561=$t /" >> gpurun_out/s3_pers_step.log 2>&1; done
LJS_GEMM_TILE2561=0 timeout -k 10 200 python bench.py --model layer >> gpurun_out/s3_pers_step.log 2>&1
