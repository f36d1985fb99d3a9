set -e
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r2gs.txt
: > $o
for i in 1 2; do
for g in 1 2 4; do
  for m in "" "--batch-per-gpu 8"; do
    echo "G=$g $m $(timeout -k 10 200 python bench.py --steps 200 --warmup 20 --graph-steps $g $m 2>&1 | grep -o '"ms_per_step": [0-9.]*')" >> $o
  done
done
done
