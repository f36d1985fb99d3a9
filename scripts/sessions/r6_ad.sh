# round-6: where the 2-D layout's segmented capture fails under gloo ("Capture must end on the
# same stream it began on", the secondary of gpurun_out/r6ab): the 2-D mesh as the headline of a
# 2-rank gloo job on the one GPU, capture cuts traced
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$PWD/gpurun_out/r6ad
mkdir -p $O
export LJS_DIST_BACKEND=gloo LJS_GRAPH_CUT_TRACE=1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29611 bench.py --gpus 2 --mesh 2d --secondary off --steps 3 --warmup 1 --min-warmup 1 > $O/gloo2_2d.txt 2>&1
echo "rc=$?" >> $O/rc.log
echo done
