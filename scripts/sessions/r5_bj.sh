# host-side cost of a graph replay at the driver shape: HIP API trace (hipGraphLaunch durations,
# first-kernel latency after the launch call); only the summary is kept (the database is large)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r5bj
mkdir -p $O
cd /tmp && timeout -k 10 300 rocprofv3 --sys-trace -d /tmp/r5bj_sys -o run -- python3 $R/bench.py --steps 20 --warmup 5 > $O/sys.log 2>&1 &&
cd $R && python scripts/api_gaps.py $(ls /tmp/r5bj_sys/*/run_results.db /tmp/r5bj_sys/run_results.db 2>/dev/null | head -1) > $O/api_gaps.txt 2>&1 && echo done
