# single-launch slab weight sweep on the fake-4 dp rehearsal: W = 4 (default) vs 8 vs 12, x3
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r5bq
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
F4="WORLD_SIZE=4 RANK=0 LOCAL_RANK=0 LJS_DIST_BACKEND=fake MASTER_ADDR=127.0.0.1"
for i in 1 2 3; do
  for w in 4 8 12; do
    p=$((29800 + 10 * w + i))
    step $O/f4_w${w}_$i.txt env $F4 LJS_DW_SINGLE_TRAFFIC_W=$w MASTER_PORT=$p timeout -k 10 200 python bench.py --gpus 4 --mesh dp --secondary off --steps 20 --warmup 5
  done
done
echo done
