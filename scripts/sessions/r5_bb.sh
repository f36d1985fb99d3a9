# the next step's input cast run by the optimizer launch's extra blocks (single-process multi-step
# graphs): precast / Adam tests, then B=64 and B=8 x3 interleaved vs LJS_OPT_PRECAST=0, B=8 trace
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r5bb
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
step $O/tests.txt timeout -k 10 700 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/ -k "prefetch or precast or adam or deferred or e2e"
for rep in 1 2 3; do
  step $O/b64_opt_$rep.txt timeout -k 10 300 python bench.py
  LJS_OPT_PRECAST=0 step $O/b64_fwd_$rep.txt timeout -k 10 300 python bench.py
  step $O/b8_opt_$rep.txt timeout -k 10 300 python bench.py --batch-per-gpu 8
  LJS_OPT_PRECAST=0 step $O/b8_fwd_$rep.txt timeout -k 10 300 python bench.py --batch-per-gpu 8
done
cd /tmp && step $O/prof_b8.txt timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof_b8 -o run -- python $R/bench.py --batch-per-gpu 8 --steps 20 --warmup 5
echo done
