# the single-launch slab weight on the 2-D rehearsal (fake-4, dp2 x tp2): W=4 (default) vs 1, x2
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r5bp
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
F4="WORLD_SIZE=4 RANK=0 LOCAL_RANK=0 LJS_DIST_BACKEND=fake MASTER_ADDR=127.0.0.1"
for i in 1 2; do
  step $O/f4_2d_w4_$i.txt env $F4 MASTER_PORT=2993$i timeout -k 10 200 python bench.py --gpus 4 --mesh 2d --steps 20 --warmup 5
  step $O/f4_2d_w1_$i.txt env $F4 LJS_DW_SINGLE_TRAFFIC_W=1 MASTER_PORT=2994$i timeout -k 10 200 python bench.py --gpus 4 --mesh 2d --steps 20 --warmup 5
done
echo done
