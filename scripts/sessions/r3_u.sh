cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r3u
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; if [ $rc -ne 0 ]; then echo "rc=$rc: $*" >> $O/rc.log; case $rc in 1|2) ;; *) exit $rc;; esac; fi; }
export LJS_DIST_BACKEND=gloo LJS_P2P=1 LJS_P2P_MAX_KB=65536 LJS_COMM_TIMEOUT_S=90
step $O/cuts.log env LJS_GRAPH_CUT_TRACE=1 timeout -k 10 200 python bench.py --gpus 2 --mesh 1x2 --steps 8 --warmup 2 --batch-per-gpu 8 --graph-steps 1
step $O/tests.log timeout -k 10 300 python -u -m pytest -x -v --timeout 280 --timeout-method thread tests/test_rehearsal_gpu.py -k "p2p_single_graph"
[ -s $O/rc.log ] && exit 1
step $O/tp2.log timeout -k 10 200 python bench.py --gpus 2 --mesh 1x2 --steps 16 --warmup 4 --batch-per-gpu 8 --graph-steps 1
step $O/tp2_pf.log env LJS_QKV_PREFETCH=1 timeout -k 10 200 python bench.py --gpus 2 --mesh 1x2 --steps 16 --warmup 4 --batch-per-gpu 8 --graph-steps 1
cd /tmp
step $O/prof_tp2_pf.log env LJS_QKV_PREFETCH=1 timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof_tp2_pf -- python3 $R/bench.py --gpus 2 --mesh 1x2 --steps 8 --warmup 2 --batch-per-gpu 8 --graph-steps 1
echo done
