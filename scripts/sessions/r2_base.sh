set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 200 python bench.py --steps 50 --warmup 10 > gpurun_out/r2b_bench64.log 2>&1
timeout -k 10 200 python bench.py --steps 200 --warmup 20 --batch-per-gpu 8 > gpurun_out/r2b_bench8.log 2>&1
timeout -k 10 200 python bench.py --steps 50 --warmup 10 --model layer > gpurun_out/r2b_layer.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r2b_prof8 -o prof -- python bench.py --steps 100 --warmup 10 --batch-per-gpu 8 > gpurun_out/r2b_prof8.log 2>&1
