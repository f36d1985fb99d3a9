set -e
cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_distributed_gpu.py -x -q --timeout 200 --timeout-method thread -k "adam or dp or distributed or slab" > gpurun_out/dp1_tests.log 2>&1
timeout -k 10 200 python bench.py --steps 50 --warmup 10 > gpurun_out/dp1_bench1.log 2>&1
LJS_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr=127.0.0.1 --master-port=29541 bench.py --gpus 2 --steps 20 --warmup 5 --batch-per-gpu 16 > gpurun_out/dp1_bench2.log 2>&1
