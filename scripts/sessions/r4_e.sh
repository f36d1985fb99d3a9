# aten-level origin of the stray kernels in the fake-4 2-D step (eager, one traced step)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r4e
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then case $rc in 1|2) ;; *) exit $rc;; esac; fi; }
F4="WORLD_SIZE=4 RANK=0 LOCAL_RANK=0 LJS_DIST_BACKEND=fake MASTER_ADDR=127.0.0.1"
step $O/trace_2d.log env $F4 MASTER_PORT=29691 LJS_ATEN_TRACE=$O/aten_2d.txt timeout -k 10 300 python bench.py --gpus 4 --mesh 2d --steps 2 --warmup 2 --min-warmup 0
step $O/trace_2d_fp8.log env $F4 MASTER_PORT=29692 LJS_ATEN_TRACE=$O/aten_2d_fp8.txt timeout -k 10 300 python bench.py --gpus 4 --mesh 2d --model layer --fp8 --steps 2 --warmup 2 --min-warmup 0
step $O/trace_dp.log env $F4 MASTER_PORT=29693 LJS_ATEN_TRACE=$O/aten_dp.txt timeout -k 10 300 python bench.py --gpus 4 --mesh dp --steps 2 --warmup 2 --min-warmup 0
echo done
