# fake-4 2-D step after the glue fixes: aten/glue trace (pack launches), kernel table, bench lines
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r4g
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then case $rc in 1|2) ;; *) exit $rc;; esac; fi; }
step $O/test_box.log timeout -k 10 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "box_slice or dropout"
F4="WORLD_SIZE=4 RANK=0 LOCAL_RANK=0 LJS_DIST_BACKEND=fake MASTER_ADDR=127.0.0.1"
step $O/trace_2d.log env $F4 MASTER_PORT=29701 LJS_ATEN_TRACE=$O/aten_2d.txt timeout -k 10 300 python bench.py --gpus 4 --mesh 2d --steps 2 --warmup 2 --min-warmup 0
step $O/fake4_2d.log env $F4 MASTER_PORT=29702 timeout -k 10 300 python bench.py --gpus 4 --mesh 2d --steps 20 --warmup 5
step $O/fake4_dp.log env $F4 MASTER_PORT=29703 timeout -k 10 300 python bench.py --gpus 4 --mesh dp --steps 20 --warmup 5
cd /tmp
export WORLD_SIZE=4 RANK=0 LOCAL_RANK=0 LJS_DIST_BACKEND=fake MASTER_ADDR=127.0.0.1
step $O/prof_2d.log env MASTER_PORT=29704 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_2d -o run -- python3 $R/bench.py --gpus 4 --mesh 2d --steps 16 --warmup 4
step $O/prof_dp.log env MASTER_PORT=29705 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_dp -o run -- python3 $R/bench.py --gpus 4 --mesh dp --steps 16 --warmup 4
echo done
