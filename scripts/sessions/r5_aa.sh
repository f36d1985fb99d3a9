# Adam count increments deferred to one launch per capture segment: tests, then bench A/B
# (LJS_ADAM_DEFER_INC=0 / 1) at B=8 and B=64 (driver shape), x3 interleaved
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r5aa
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
step $O/tests.txt timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu -k "adam or jit_graph or capture or train" tests/
for rep in 1 2 3; do
  for b in 8 64; do
    LJS_ADAM_DEFER_INC=0 step $O/b${b}_off_$rep.txt timeout -k 10 300 python bench.py --batch-per-gpu $b --steps 20 --warmup 5
    step $O/b${b}_on_$rep.txt timeout -k 10 300 python bench.py --batch-per-gpu $b --steps 20 --warmup 5
  done
done
echo done
