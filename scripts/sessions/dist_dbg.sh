cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD LJS_PLATFORM=gpu LJS_DIST_BACKEND=gloo LJS_HANG_DUMP_S=100
timeout -k 10 150 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr=127.0.0.1 --master-port=29533 scripts/dp_check.py /tmp/r2.npz 3 1 > gpurun_out/d2.log 2>&1; echo "rc=$?" >> gpurun_out/d2.log
unset LJS_HANG_DUMP_S
timeout -k 10 400 python -m pytest tests/test_distributed_gpu.py -x -q > gpurun_out/dist.log 2>&1; echo "rc=$?" >> gpurun_out/dist.log
