set -e
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r2attnab.txt
: > $o
for cfg in "X=1" "LJS_ATTN_FWD_RES=16" "LJS_ATTN_FWD_RES=116" "LJS_ATTN_FWD_RES=108" "LJS_ATTN_BWD_FUSED=0" "LJS_ATTN_PRIO=0"; do
  for m in "" "--batch-per-gpu 8"; do
    echo "$cfg $m $(env $cfg timeout -k 10 200 python bench.py --steps 100 --warmup 20 $m 2>&1 | grep -o '"ms_per_step": [0-9.]*')" >> $o
  done
done
