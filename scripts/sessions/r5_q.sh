# after removing the 4-wave wide GEMM tiles and the Adam thread / ticket-form knobs: GEMM + Adam GPU
# tests; then the graph-size sweep with the JSON's peak reserved memory (G = 1 / 5 / 20)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r5q
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
step $O/tests.txt timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu -k "adam or gemm or lean" tests/
for g in 1 5 20; do
  step $O/bench_g$g.txt timeout -k 10 300 python bench.py --steps 20 --warmup 5 --graph-steps $g
done
echo done
