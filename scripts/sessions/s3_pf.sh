set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
LJS_GEMM_PF=2 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x -k "gemm" --timeout 120 --timeout-method thread > gpurun_out/s3_pf_tests.log 2>&1
for pf in 0 1 2 3 4; do
  for cfg in "qkv 2561" "out 1282" "dattn 1282" "dwall_slabs 1282 8" "dwo_slabs 1282 16"; do
    LJS_GEMM_PF=$pf timeout -k 10 60 python scripts/gemm_one.py $cfg | sed "s/^/pf=$pf /" >> gpurun_out/s3_pf_times.log 2>&1
  done
  LJS_GEMM_PF=$pf timeout -k 10 200 python bench.py | sed "s/^/pf=$pf /" >> gpurun_out/s3_pf_bench.log 2>&1
done
