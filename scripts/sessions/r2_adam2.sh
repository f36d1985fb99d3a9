set -e
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r2adam2.txt
: > $o
for i in 1 2 3; do
for r in 64 32 16; do
  for m in "" "--batch-per-gpu 8"; do
    echo "rows=$r $m $(LJS_ADAM_ROWS=$r timeout -k 10 200 python bench.py --steps 200 --warmup 20 $m 2>&1 | grep -o '"ms_per_step": [0-9.]*')" >> $o
  done
done
done
