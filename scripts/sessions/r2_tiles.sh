set -e
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r2tiles.txt
: > $o
for i in 1 2; do
for cfg in "X=1" "LJS_GEMM_TILE2561=0" "LJS_GEMM_TILE1602=0" "LJS_DMA_BPC=1"; do
  echo "$cfg $(env $cfg timeout -k 10 200 python bench.py --steps 100 --warmup 20 2>&1 | grep -o '"ms_per_step": [0-9.]*')" >> $o
done
done
