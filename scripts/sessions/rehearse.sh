set -e
cd "$GRAFT_REPO_ROOT"
for w in 2 8; do
WORLD_SIZE=$w RANK=0 LOCAL_RANK=0 LJS_DIST_BACKEND=fake MASTER_PORT=29555 timeout -k 10 200 python bench.py --steps 50 --warmup 10 > gpurun_out/reh_w$w.log 2>&1
done
WORLD_SIZE=8 RANK=0 LOCAL_RANK=0 LJS_DIST_BACKEND=fake LJS_GRAD_BUCKET_MB=64 MASTER_PORT=29555 timeout -k 10 200 python bench.py --steps 50 --warmup 10 > gpurun_out/reh_w8_b64.log 2>&1
WORLD_SIZE=8 RANK=0 LOCAL_RANK=0 LJS_DIST_BACKEND=fake LJS_OVERLAP_GRAD_REDUCE=0 MASTER_PORT=29555 timeout -k 10 200 python bench.py --steps 50 --warmup 10 > gpurun_out/reh_w8_noov.log 2>&1
