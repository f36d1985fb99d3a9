# round-6: the driver's multi-rank launch form (torch.distributed.run, one process per rank) with
# real data movement: N ranks share the box's one GPU over gloo (RCCL refuses two ranks on one
# device).  Checks the N > 1 bench path end to end: comm_detail, the all-reduce probe, the 2-D
# secondary.  Timings here carry no scaling meaning (the ranks share one GPU).
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$PWD/gpurun_out/r6ab
mkdir -p $O
export LJS_DIST_BACKEND=gloo
for n in 2 4; do
  timeout -k 10 420 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29600 + n)) bench.py --gpus $n --steps 10 --warmup 3 > $O/gloo$n.txt 2>&1
  rc=$?
  echo "n=$n rc=$rc" >> $O/rc.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
echo done
