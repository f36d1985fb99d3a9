set -e
cd "$GRAFT_REPO_ROOT"
PYTHONPATH=$PWD LJS_PLATFORM=gpu timeout -k 10 300 python cases/case6_attention.py > gpurun_out/m_case6.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_b8fwd" -- python3 "$GRAFT_REPO_ROOT/bench.py" --batch-per-gpu 8 --mode fwd --steps 50 --warmup 5 > "$GRAFT_REPO_ROOT/gpurun_out/prof_b8fwd.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_b8" -- python3 "$GRAFT_REPO_ROOT/bench.py" --batch-per-gpu 8 --steps 50 --warmup 5 > "$GRAFT_REPO_ROOT/gpurun_out/prof_b8.log" 2>&1
