# slab-traffic weight of the single weight-gradient pick (the multi-process dp path, where the pair
# does not apply and slab_reduce reads every slab): fake-4 dp rehearsal x3, W=1 (default) vs W=4
# (dW_o 16 splits instead of 24), plus N=1 B=64 with W=4
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r5bm2
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
F4="WORLD_SIZE=4 RANK=0 LOCAL_RANK=0 LJS_DIST_BACKEND=fake MASTER_ADDR=127.0.0.1"
for i in 1 2 3; do
  step $O/f4_w1_$i.txt env $F4 MASTER_PORT=2998$i timeout -k 10 200 python bench.py --gpus 4 --mesh dp --secondary off --steps 20 --warmup 5
  step $O/f4_w4_$i.txt env $F4 LJS_DW_TRAFFIC_W=4 MASTER_PORT=2999$i timeout -k 10 200 python bench.py --gpus 4 --mesh dp --secondary off --steps 20 --warmup 5
done
echo done
