cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r3n
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; if [ $rc -ne 0 ]; then echo "rc=$rc: $*" >> $O/rc.log; case $rc in 1|2) ;; *) exit $rc;; esac; fi; }
F4="WORLD_SIZE=4 RANK=0 LOCAL_RANK=0 LJS_DIST_BACKEND=fake MASTER_ADDR=127.0.0.1"
step $O/tests.log timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_gpu_e2e.py -k "attention or attn or block_gpu or ring"
cd /tmp
step $O/kt_bwd64.log timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/kt_bwd64 -o run -- python3 $R/scripts/attn_one.py bwd 64 256 8 10
step $O/kt_bwd2d.log timeout -k 10 120 python3 $R/scripts/attn_layout.py
step $O/prof_layer8.log timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_layer8 -o run -- python3 $R/bench.py --model layer --fp8 --steps 24 --warmup 6
cd $R
for i in 1 2; do
  step $O/b64_$i.log timeout -k 10 200 python bench.py
  step $O/fake4_2d_$i.log env $F4 MASTER_PORT=2967$i timeout -k 10 300 python bench.py --gpus 4 --mesh 2d
done
step $O/fake4_dp.log env $F4 MASTER_PORT=29692 timeout -k 10 300 python bench.py --gpus 4 --mesh dp
echo done
