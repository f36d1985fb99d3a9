set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for a in "--seq 4096 --batch-per-gpu 4" "--seq 1024 --batch-per-gpu 16" "--seq 4096 --batch-per-gpu 4 --mode fwd"; do
  echo "$a $(timeout -k 10 200 python bench.py --steps 32 --warmup 8 $a | tail -1)" >> gpurun_out/r2c_long.log
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r2c_long4k -o prof -- python bench.py --steps 16 --warmup 8 --seq 4096 --batch-per-gpu 4 > /dev/null 2>&1
