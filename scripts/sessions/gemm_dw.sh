set -e
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q -k gemm > gpurun_out/kern.log 2>&1
for c in "dwqkv 1282 4" "dwqkv 1282 8" "dwqkv 1282 16" "dwqkv 1284 8" "dwqkv 1284 4" "dwo 1282 8" "dwo 1282 16" "dwo 1284 16" "dwo 1284 8"; do
  timeout -k 10 60 python scripts/gemm_one.py $c
done > gpurun_out/one.log 2>&1
