# round-6: the driver's launch form at N = 4 and 8 ranks sharing the box's one GPU over gloo,
# after the segmented-capture fix: dp headline + the 2-D (N/2, 2) secondary, functional check
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$PWD/gpurun_out/r6af
mkdir -p $O
export LJS_DIST_BACKEND=gloo
for n in 4 8; do
  timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29800 + n)) bench.py --gpus $n --steps 10 --warmup 3 > $O/gloo$n.txt 2>&1
  rc=$?
  echo "n=$n rc=$rc" >> $O/rc.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
echo done
