set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/s3_sc1_tests.log 2>&1
for sc in 0 1; do
  for cfg in "qkv 2561" "out 1282" "dattn 1282" "dwall_slabs 1282 8" "dwo_slabs 1282 16"; do
    LJS_GEMM_SC1=$sc timeout -k 10 60 python scripts/gemm_one.py $cfg | sed "s/^/sc1=$sc /" >> gpurun_out/s3_sc1_times.log 2>&1
  done
  LJS_GEMM_SC1=$sc timeout -k 10 200 python bench.py | sed "s/^/sc1=$sc /" >> gpurun_out/s3_sc1_bench.log 2>&1
done
