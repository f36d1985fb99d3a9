# Adam at 32-row tiles by default (64 with MX shadows): Adam / fp8 / e2e GPU tests, then B=64 and
# B=8 x2 and the fp8 layer once
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r5ak
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
step $O/tests.txt timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/ -k "adam or fp8 or mx or e2e or shadow or optim or deferred or grouped"
for rep in 1 2; do
  step $O/b64_$rep.txt timeout -k 10 300 python bench.py
  step $O/b8_$rep.txt timeout -k 10 300 python bench.py --batch-per-gpu 8
done
step $O/fp8_layer.txt timeout -k 10 300 python bench.py --model layer --fp8
echo done
