set -e
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r2dws.txt
: > $o
for i in 1 2 3; do
for t in 644 12884; do
  echo "tile=$t $(LJS_DW_SMALL_TILE=$t timeout -k 10 200 python bench.py --steps 200 --warmup 20 --batch-per-gpu 8 2>&1 | grep -o '"ms_per_step": [0-9.]*')" >> $o
done
done
