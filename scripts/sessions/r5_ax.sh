# the next step's input cast queued before the data-parallel gradient join (LJS_PRECAST=join):
# bit-exact 2-rank test, e2e precast test, fake-4 dp rehearsal x2 (join vs 0), 1-GPU bench
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r5ax
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
step $O/tests.txt timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_distributed_gpu.py tests/test_gpu_e2e.py tests/test_rehearsal_gpu.py -k "precast or dp2 or dp8 or prefetch"
F4="WORLD_SIZE=4 RANK=0 LOCAL_RANK=0 LJS_DIST_BACKEND=fake MASTER_ADDR=127.0.0.1"
for i in 1 2; do
  step $O/f4_dp_join_$i.txt env $F4 MASTER_PORT=2994$i timeout -k 10 200 python bench.py --gpus 4 --mesh dp --secondary off --steps 20 --warmup 5
  step $O/f4_dp_off_$i.txt env $F4 LJS_PRECAST=0 MASTER_PORT=2995$i timeout -k 10 200 python bench.py --gpus 4 --mesh dp --secondary off --steps 20 --warmup 5
done
step $O/b64.txt timeout -k 10 300 python bench.py
echo done
