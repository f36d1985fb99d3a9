cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3dbg; mkdir -p $O
WORLD_SIZE=4 RANK=0 LOCAL_RANK=0 LJS_DIST_BACKEND=fake MASTER_ADDR=127.0.0.1 MASTER_PORT=29650 LJS_SHADOW_TRACE=1 timeout -k 10 200 python bench.py --gpus 4 --mesh 2d --steps 3 --warmup 3 --no-graph --batch-per-gpu 8 > $O/fake2d_trace.log 2>&1
LJS_SHADOW_TRACE=1 timeout -k 10 200 python bench.py --steps 3 --warmup 3 --no-graph --batch-per-gpu 8 > $O/dp_trace.log 2>&1
echo done
