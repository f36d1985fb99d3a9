set -e
cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -m pytest tests/test_kernels_gpu.py tests/test_gpu_e2e.py -x -q > gpurun_out/kern.log 2>&1
timeout -k 10 200 python bench.py --steps 50 --warmup 10 > gpurun_out/bench.log 2>&1
LJS_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr=127.0.0.1 --master-port=29541 bench.py --gpus 2 --steps 20 --warmup 5 --batch-per-gpu 16 > gpurun_out/bench2.log 2>&1
