# the per-replay completion event made lazy (graphs._note_replay): driver shape x3 interleaved vs
# LJS_REPLAY_EVENT=1, plus a kernel trace for the inter-graph gaps
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r5ar
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
for rep in 1 2 3; do
  step $O/b64_lazy_$rep.txt timeout -k 10 300 python bench.py --steps 20 --warmup 5
  LJS_REPLAY_EVENT=1 step $O/b64_event_$rep.txt timeout -k 10 300 python bench.py --steps 20 --warmup 5
done
cd /tmp && step $O/prof_b64.txt timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof_b64 -o run -- python $R/bench.py --steps 20 --warmup 5
echo done
