cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r3v
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; if [ $rc -ne 0 ]; then echo "rc=$rc: $*" >> $O/rc.log; case $rc in 1|2) ;; *) exit $rc;; esac; fi; }
for pc in 1 0; do
  step $O/b8_pc${pc}.log env DEBUG_CLR_GRAPH_PACKET_CAPTURE=$pc timeout -k 10 200 python bench.py --batch-per-gpu 8
  step $O/b8_ea_pc${pc}.log env DEBUG_CLR_GRAPH_PACKET_CAPTURE=$pc LJS_EARLY_ADAM=1 timeout -k 10 200 python bench.py --batch-per-gpu 8
  step $O/b64_pc${pc}.log env DEBUG_CLR_GRAPH_PACKET_CAPTURE=$pc timeout -k 10 200 python bench.py
  step $O/b64_ea_pc${pc}.log env DEBUG_CLR_GRAPH_PACKET_CAPTURE=$pc LJS_EARLY_ADAM=1 timeout -k 10 200 python bench.py
done
cd /tmp
for pc in 1 0; do
  step $O/prof_b8_ea_pc${pc}.log env DEBUG_CLR_GRAPH_PACKET_CAPTURE=$pc LJS_EARLY_ADAM=1 timeout -k 10 200 rocprofv3 --kernel-trace -d $O/prof_b8_ea_pc${pc} -o run -- python3 $R/bench.py --batch-per-gpu 8 --steps 16 --warmup 4
done
cd $R
export LJS_DIST_BACKEND=gloo LJS_P2P=1 LJS_P2P_MAX_KB=65536 LJS_COMM_TIMEOUT_S=90
step $O/tp2_pf_pc0.log env DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 LJS_QKV_PREFETCH=1 timeout -k 10 200 python bench.py --gpus 2 --mesh 1x2 --steps 16 --warmup 4 --batch-per-gpu 8 --graph-steps 1
cd /tmp
step $O/prof_tp2_pf_pc0.log env DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 LJS_QKV_PREFETCH=1 timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof_tp2_pf_pc0 -- python3 $R/bench.py --gpus 2 --mesh 1x2 --steps 8 --warmup 2 --batch-per-gpu 8 --graph-steps 1
echo done
