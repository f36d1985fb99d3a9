set -e
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -m pytest tests/test_gpu_e2e.py -x -q -k "jit" > gpurun_out/e2e.log 2>&1
timeout -k 10 200 python bench.py --batch-per-gpu 8 --mode fwd --steps 200 --warmup 20 > gpurun_out/m_fwd8.log 2>&1
timeout -k 10 200 python bench.py --batch-per-gpu 8 --steps 200 --warmup 20 > gpurun_out/m_train8.log 2>&1
timeout -k 10 200 python bench.py --steps 100 --warmup 10 > gpurun_out/m_train64.log 2>&1
