# HIP runtime knobs vs the ~14 us GPU idle between graph replays (driver shape, B=64 / B=8, x2)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r5aq
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
for rep in 1 2; do
  step $O/b64_base_$rep.txt timeout -k 10 300 python bench.py --steps 20 --warmup 5
  DEBUG_HIP_GRAPH_BATCH_SIZE=1024 step $O/b64_gbatch1024_$rep.txt timeout -k 10 300 python bench.py --steps 20 --warmup 5
  DEBUG_HIP_GRAPH_BATCH_SIZE=4 step $O/b64_gbatch4_$rep.txt timeout -k 10 300 python bench.py --steps 20 --warmup 5
  ROC_SYSTEM_SCOPE_SIGNAL=0 step $O/b64_agentsig_$rep.txt timeout -k 10 300 python bench.py --steps 20 --warmup 5
  HIP_FORCE_DEV_KERNARG=1 step $O/b64_devkernarg_$rep.txt timeout -k 10 300 python bench.py --steps 20 --warmup 5
  ROC_ACTIVE_WAIT_TIMEOUT=0 step $O/b64_nowait_$rep.txt timeout -k 10 300 python bench.py --steps 20 --warmup 5
done
echo done
