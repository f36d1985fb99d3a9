# Adam tile-height balance relative to the lightest slab gradient: tests, then B=8 / B=64 A/B
# (LJS_ADAM_BALANCE=0 / 1); 2-D glue trace (r5_w) afterwards
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r5y
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
step $O/tests.txt timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu -k "adam" tests/
for rep in 1 2 3; do
  for b in 8 64; do
    LJS_ADAM_BALANCE=0 step $O/b${b}_off_$rep.txt timeout -k 10 300 python bench.py --batch-per-gpu $b
    step $O/b${b}_on_$rep.txt timeout -k 10 300 python bench.py --batch-per-gpu $b
  done
done
bash scripts/sessions/r5_w.sh
echo done
