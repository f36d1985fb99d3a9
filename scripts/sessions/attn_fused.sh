set -e
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q -k attention > gpurun_out/kern.log 2>&1
timeout -k 10 120 python scripts/attn_bench.py > gpurun_out/attn.log 2>&1
timeout -k 10 120 python scripts/attn_bench.py 8 256 8 64 >> gpurun_out/attn.log 2>&1
timeout -k 10 300 python -m pytest tests/test_gpu_e2e.py -x -q > gpurun_out/e2e.log 2>&1
timeout -k 10 200 python bench.py --steps 50 --warmup 10 > gpurun_out/bench.log 2>&1
