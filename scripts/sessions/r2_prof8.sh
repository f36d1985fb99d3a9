set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
o=gpurun_out/r2prof8.txt
: > $o
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r2p8_b8 -o prof -- python bench.py --steps 20 --warmup 5 --batch-per-gpu 8 > gpurun_out/r2p8_b8.log 2>&1
for m in "--model layer" "--model layer --fp8" "--model ff" "--model ff --fp8" "--model fsdp"; do
  echo "$m $(timeout -k 10 200 python bench.py --steps 100 --warmup 20 $m 2>&1 | grep -o '"ms_per_step": [0-9.]*')" >> $o
done
