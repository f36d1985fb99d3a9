set -e
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_native_rccl_gpu.py tests/test_rehearsal_gpu.py -x -v --timeout 280 --timeout-method thread > gpurun_out/native1_tests.log 2>&1 || true
for w in 2 8; do
WORLD_SIZE=$w RANK=0 LOCAL_RANK=0 LJS_DIST_BACKEND=fake MASTER_PORT=29555 timeout -k 10 200 python bench.py --gpus $w --steps 50 --warmup 10 > gpurun_out/reh2_w$w.log 2>&1
done
