set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x -k "attention" --timeout 120 --timeout-method thread > gpurun_out/s3_pa_tests.log 2>&1
for r in 8 108 116; do
  LJS_ATTN_FWD_RES=$r timeout -k 10 100 python scripts/attn_bench.py | sed "s/^/res=$r /" >> gpurun_out/s3_pa_bench.log 2>&1
  LJS_ATTN_FWD_RES=$r timeout -k 10 200 python bench.py | sed "s/^/res=$r /" >> gpurun_out/s3_pa_step.log 2>&1
done
