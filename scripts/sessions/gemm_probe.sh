set -e
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q -k gemm > gpurun_out/kern.log 2>&1
for c in "dwo 1282 8" "dwo 1282 16" "dwo 1284 8" "dwo 1284 16" "dwqkv 1282 4" "dwqkv 1282 8" "dwqkv 1284 4" "dwqkv 1284 8" "qkv 2561" "qkv 1282" "qkv 1284" "out 2561" "out 1282" "out 1284" "dattn 2561" "dattn 1282" "dattn 1284"; do
  timeout -k 10 60 python scripts/gemm_one.py $c
done > gpurun_out/one.log 2>&1
