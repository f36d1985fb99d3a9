# the Adam in-kernel count ticket removed: Adam / precast / deferred / e2e GPU tests, fp8 layer and
# B=64 / B=8 benches
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r5bk
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
step $O/tests.txt timeout -k 10 700 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/ -k "adam or prefetch or precast or deferred or e2e or optim or fp8 or shadow"
step $O/b64.txt timeout -k 10 300 python bench.py
step $O/b8.txt timeout -k 10 300 python bench.py --batch-per-gpu 8
step $O/fp8.txt timeout -k 10 300 python bench.py --model layer --fp8
echo done
