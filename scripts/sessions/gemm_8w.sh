set -e
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q -k gemm > gpurun_out/kern.log 2>&1
for c in "dwqkv 1282 8" "dwqkv 12883 8" "dwqkv 12884 8" "dwqkv 12883 4" "dwqkv 12884 4" "dwo 1282 16" "dwo 12883 16" "dwo 12884 16" "dwo 12884 8" "qkv 1282" "qkv 12883" "qkv 12884" "out 1282" "out 12883" "dattn 1282" "dattn 12883"; do
  timeout -k 10 60 python scripts/gemm_one.py $c
done > gpurun_out/one.log 2>&1
