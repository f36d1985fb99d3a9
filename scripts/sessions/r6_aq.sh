# round-6: the driver's scaling command shape rehearsed on one GPU (fake backend, rank 0 of N) on
# the fused-attention build: N = 2 / 4 / 8 (collectives move nothing; checks the N > 1 path runs
# and prints its comm_detail / secondary objects)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r6aq
mkdir -p $O
for n in 2 4 8; do
  WORLD_SIZE=$n RANK=0 LOCAL_RANK=0 LJS_DIST_BACKEND=fake MASTER_ADDR=127.0.0.1 MASTER_PORT=2995$n timeout -k 10 300 python bench.py --gpus $n --steps 20 --warmup 5 > $O/fake$n.log 2>&1 || exit 3
done
echo done
