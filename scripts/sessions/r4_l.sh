# MX-fp8 shadow gather for the 2-D FF block: tests, glue trace, rehearsal bench lines, kernel table
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r4l
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then case $rc in 1|2) ;; *) exit $rc;; esac; fi; }
step $O/tests.log timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_e2e.py -k "fp8"
if grep -q " failed\|[0-9] error" $O/tests.log; then echo "tests failed"; tail -40 $O/tests.log; exit 1; fi
F4="WORLD_SIZE=4 RANK=0 LOCAL_RANK=0 LJS_DIST_BACKEND=fake MASTER_ADDR=127.0.0.1"
step $O/trace_2d_fp8.log env $F4 MASTER_PORT=29741 LJS_ATEN_TRACE=$O/aten_2d_fp8.txt timeout -k 10 300 python bench.py --gpus 4 --mesh 2d --model layer --fp8 --steps 2 --warmup 2 --min-warmup 0
for i in 1 2; do
step $O/fake4_2d_fp8_$i.log env $F4 MASTER_PORT=2974$((1+i)) timeout -k 10 300 python bench.py --gpus 4 --mesh 2d --model layer --fp8 --steps 20 --warmup 5
step $O/fake4_dp_fp8_$i.log env $F4 MASTER_PORT=2975$((1+i)) timeout -k 10 300 python bench.py --gpus 4 --mesh dp --model layer --fp8 --steps 20 --warmup 5
step $O/layer_fp8_$i.log timeout -k 10 200 python bench.py --model layer --fp8 --steps 20 --warmup 5
step $O/fake4_2d_$i.log env $F4 MASTER_PORT=2976$((1+i)) timeout -k 10 300 python bench.py --gpus 4 --mesh 2d --steps 20 --warmup 5
step $O/fake4_dp_$i.log env $F4 MASTER_PORT=2977$((1+i)) timeout -k 10 300 python bench.py --gpus 4 --mesh dp --steps 20 --warmup 5
done
cd /tmp
export WORLD_SIZE=4 RANK=0 LOCAL_RANK=0 LJS_DIST_BACKEND=fake MASTER_ADDR=127.0.0.1
step $O/prof_2d_fp8.log env MASTER_PORT=29781 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_2d_fp8 -o run -- python3 $R/bench.py --gpus 4 --mesh 2d --model layer --fp8 --steps 16 --warmup 4
cd $R
step $O/mfma_rate.log timeout -k 10 120 ./scripts/mfma_rate
echo done
