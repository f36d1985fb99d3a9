set -e
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -m pytest tests/test_p2p_gpu.py -x -q > gpurun_out/p2p.log 2>&1
