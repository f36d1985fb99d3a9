cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r3k
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; if [ $rc -ne 0 ]; then echo "rc=$rc: $*" >> $O/rc.log; case $rc in 1|2) ;; *) exit $rc;; esac; fi; }
F4="WORLD_SIZE=4 RANK=0 LOCAL_RANK=0 LJS_DIST_BACKEND=fake MASTER_ADDR=127.0.0.1"
step $O/tests.log timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_gpu_e2e.py -k "fp8 or quant or mx or local_first or block_gpu or layer"
step $O/fp8_tiles.log timeout -k 10 300 python scripts/fp8_tiles.py 20 1282,256160
for i in 1 2; do
  step $O/layer8_$i.log timeout -k 10 200 python bench.py --model layer --fp8
  step $O/fake4_2d_p1_$i.log env $F4 MASTER_PORT=2967$i LJS_QKV_PREFETCH=1 timeout -k 10 300 python bench.py --gpus 4 --mesh 2d
  step $O/fake4_2d_p0_$i.log env $F4 MASTER_PORT=2968$i LJS_QKV_PREFETCH=0 timeout -k 10 300 python bench.py --gpus 4 --mesh 2d
  step $O/v2x2_p1_$i.log env LJS_NUM_DEVICES=4 LJS_QKV_PREFETCH=1 timeout -k 10 300 python bench.py --mesh 2x2
  step $O/v2x2_p0_$i.log env LJS_NUM_DEVICES=4 LJS_QKV_PREFETCH=0 timeout -k 10 300 python bench.py --mesh 2x2
done
step $O/fake4_dp.log env $F4 MASTER_PORT=29692 timeout -k 10 300 python bench.py --gpus 4 --mesh dp
step $O/replay_2d.log env $F4 MASTER_PORT=29693 LJS_REPLAY_TRACE=1 timeout -k 10 300 python bench.py --gpus 4 --mesh 2d --steps 16 --warmup 16
cd /tmp
step $O/prof_layer8.log timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_layer8 -o run -- python3 $R/bench.py --model layer --fp8 --steps 24 --warmup 6
step $O/prof_v2x2.log env LJS_NUM_DEVICES=4 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_v2x2 -o run -- python3 $R/bench.py --mesh 2x2 --steps 24 --warmup 6
echo done
