# round-6: graph length at the driver shape on the fused build (G = steps per captured graph)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r6x
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
for rep in 1 2 3; do
  for g in 8 4 10 20; do
    step $O/g${g}_$rep.txt timeout -k 10 300 python bench.py --steps 20 --warmup 5 --graph-steps $g
  done
done
for f in $O/g*_*.txt; do echo "$(basename $f) $(grep -o '"ms_per_step": [0-9.]*' $f) $(grep -o '"steps_per_graph": [0-9]*' $f)"; done > $O/lines.txt
echo done
