# kernel-trace profile of the 1-GPU bench step (argument: output tag)
set -e
TAG=${1:-prof}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/$TAG" -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 5 > "$GRAFT_REPO_ROOT/gpurun_out/$TAG.log" 2>&1
