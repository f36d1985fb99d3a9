set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof6 -o run -- python bench.py --steps 25 --warmup 5 > gpurun_out/prof6.log 2>&1
timeout -k 10 200 python bench.py --steps 50 --warmup 10 --batch-per-gpu 8 > gpurun_out/bench_b8.log 2>&1
timeout -k 10 200 python bench.py --steps 50 --warmup 10 --mode fwd > gpurun_out/bench_fwd.log 2>&1
