# the single-launch slab weight as the default (LJS_DW_SINGLE_TRAFFIC_W=4): fake-4 dp x3 vs =1,
# N=1 B=64 / B=8 / bf16 layer sanity, pick / grouping GPU tests
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r5bn
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
step $O/tests.txt timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/ -k "gemm_group or grouped or deferred or slab or e2e or dp2"
F4="WORLD_SIZE=4 RANK=0 LOCAL_RANK=0 LJS_DIST_BACKEND=fake MASTER_ADDR=127.0.0.1"
for i in 1 2 3; do
  step $O/f4_w4_$i.txt env $F4 MASTER_PORT=2990$i timeout -k 10 200 python bench.py --gpus 4 --mesh dp --secondary off --steps 20 --warmup 5
  step $O/f4_w1_$i.txt env $F4 LJS_DW_SINGLE_TRAFFIC_W=1 MASTER_PORT=2989$i timeout -k 10 200 python bench.py --gpus 4 --mesh dp --secondary off --steps 20 --warmup 5
done
step $O/b64.txt timeout -k 10 300 python bench.py
step $O/b8.txt timeout -k 10 300 python bench.py --batch-per-gpu 8
step $O/layer.txt timeout -k 10 300 python bench.py --model layer
echo done
