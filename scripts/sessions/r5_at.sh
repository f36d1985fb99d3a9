# Adam: non-MX tensors at 32-row tiles inside a 64-row (MX-shadow) launch; fp8 layer x3 vs
# LJS_ADAM_BALANCE=0 is not the same switch, so A/B against the previous build's numbers
# (r5ao: 0.5799-0.5811) plus the Adam / fp8 GPU tests
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r5at
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
step $O/tests.txt timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ -k "adam or fp8 or mx or shadow or deferred"
for rep in 1 2 3; do
  step $O/fp8_$rep.txt timeout -k 10 300 python bench.py --model layer --fp8
  LJS_ADAM_ROWS=64 step $O/fp8_rows64_$rep.txt timeout -k 10 300 python bench.py --model layer --fp8
done
echo done
