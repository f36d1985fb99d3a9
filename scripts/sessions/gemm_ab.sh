set -e
cd "$GRAFT_REPO_ROOT"
for bpc in 0 1000; do
for c in "dwqkv 1282 8" "qkv 2561" "qkv 1282" "out 2561" "out 1282" "dattn 2561" "dattn 1282"; do
  LJS_DMA_BPC=$bpc timeout -k 10 60 python scripts/gemm_one.py $c | sed "s/^/bpc=$bpc /"
done
done > gpurun_out/one.log 2>&1
