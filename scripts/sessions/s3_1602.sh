set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -q -x -k "gemm or linear or fused_output" --timeout 120 --timeout-method thread > gpurun_out/s3_1602_tests.log 2>&1
for t in 1 0; do
  LJS_GEMM_TILE1602=$t timeout -k 10 60 python scripts/gemm_one.py out 0 | sed "s/^/t1602=$t /" >> gpurun_out/s3_1602_times.log 2>&1 || true
  LJS_GEMM_TILE1602=$t timeout -k 10 200 python bench.py | sed "s/^/t1602=$t /" >> gpurun_out/s3_1602_step.log 2>&1
done
