cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r3i
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; if [ $rc -ne 0 ]; then echo "rc=$rc: $*" >> $O/rc.log; case $rc in 1|2) ;; *) exit $rc;; esac; fi; }
F4="WORLD_SIZE=4 RANK=0 LOCAL_RANK=0 LJS_DIST_BACKEND=fake MASTER_ADDR=127.0.0.1"
step $O/tests.log timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_e2e.py tests/test_rehearsal_gpu.py tests/test_distributed_gpu.py
for i in 1 2; do
  step $O/fake4_2d_h1_$i.log env $F4 MASTER_PORT=2967$i LJS_SEED_HOIST=1 timeout -k 10 300 python bench.py --gpus 4 --mesh 2d
  step $O/fake4_2d_h0_$i.log env $F4 MASTER_PORT=2968$i LJS_SEED_HOIST=0 timeout -k 10 300 python bench.py --gpus 4 --mesh 2d
  step $O/fake4_dp_$i.log env $F4 MASTER_PORT=2969$i timeout -k 10 300 python bench.py --gpus 4 --mesh dp
done
step $O/v2x2.log env LJS_NUM_DEVICES=4 timeout -k 10 300 python bench.py --mesh 2x2
cd /tmp
step $O/prof_fake4_2d.log env $F4 MASTER_PORT=29662 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_fake4_2d -o run -- python3 $R/bench.py --gpus 4 --mesh 2d --steps 24 --warmup 6
step $O/prof_v2x2.log env LJS_NUM_DEVICES=4 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_v2x2 -o run -- python3 $R/bench.py --mesh 2x2 --steps 24 --warmup 6
echo done
