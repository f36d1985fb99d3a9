set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r2b8p_prof -o prof -- python bench.py --steps 20 --warmup 5 --batch-per-gpu 8 > gpurun_out/r2b8p_prof.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r2b64p_prof -o prof -- python bench.py --steps 20 --warmup 5 > gpurun_out/r2b64p_prof.log 2>&1
