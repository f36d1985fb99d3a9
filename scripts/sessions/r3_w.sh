cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r3w
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; if [ $rc -ne 0 ]; then echo "rc=$rc: $*" >> $O/rc.log; case $rc in 1|2) ;; *) exit $rc;; esac; fi; }
for i in 1 2 3; do
  for pc in 1 0; do
    step $O/b64_pc${pc}_$i.log env DEBUG_CLR_GRAPH_PACKET_CAPTURE=$pc timeout -k 10 200 python bench.py
    step $O/b8_pc${pc}_$i.log env DEBUG_CLR_GRAPH_PACKET_CAPTURE=$pc timeout -k 10 200 python bench.py --batch-per-gpu 8
    step $O/b8g1_pc${pc}_$i.log env DEBUG_CLR_GRAPH_PACKET_CAPTURE=$pc timeout -k 10 200 python bench.py --batch-per-gpu 8 --graph-steps 1
  done
done
for pc in 1 0; do
  step $O/l8_pc${pc}.log env DEBUG_CLR_GRAPH_PACKET_CAPTURE=$pc timeout -k 10 200 python bench.py --model layer --fp8
done
echo done
