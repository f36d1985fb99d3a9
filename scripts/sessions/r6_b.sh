# round-6: GPU tests of the session's fixes (in-graph step reads, precast commit, adam), the
# per-step shader clock beside the kernel trace (slow start), and the driver-shape bench
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r6b
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
step $O/tests.txt timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu -k "multi_step or jit_graph or adam or precast" tests/
cd /tmp
step $O/ramp.log timeout -k 10 300 env LJS_CLOCK_PROBE=$O/clock.json rocprofv3 --kernel-trace -d $O/ramp -o run -- python3 $R/bench.py --steps 20 --warmup 5
step $O/ramp0.log timeout -k 10 300 env LJS_CLOCK_PROBE=$O/clock0.json rocprofv3 --kernel-trace -d $O/ramp0 -o run -- python3 $R/bench.py --steps 40 --warmup 2 --min-warmup 0
cd $R
step $O/b64.txt timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5
step $O/clk_nograph.txt timeout -k 10 300 env LJS_CLOCK_PROBE=$O/clock_plain.json python bench.py --steps 20 --warmup 5
python scripts/clock_ramp.py $O/ramp/run_results.db $O/clock.json --out $O/clock_ramp.md > /dev/null 2>&1
python scripts/clock_ramp.py $O/ramp0/run_results.db $O/clock0.json --out $O/clock_ramp0.md > /dev/null 2>&1
echo done
