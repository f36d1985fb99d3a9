# full check: GPU tests, bench, kernel profile (stops at the first failing step)
set -e
cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -m pytest tests/test_kernels_gpu.py -x -q > gpurun_out/kern.log 2>&1
timeout -k 10 500 python -m pytest tests/test_gpu_e2e.py -x -q > gpurun_out/e2e.log 2>&1
timeout -k 10 200 python bench.py --steps 50 --warmup 10 > gpurun_out/bench.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof5" -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 5 > "$GRAFT_REPO_ROOT/gpurun_out/prof5.log" 2>&1
