# side-stream early Adam and side-stream input-cast prefetch removed: the affected GPU tests,
# then B=64 / B=8 once
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r5bc
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
step $O/tests.txt timeout -k 10 700 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/ -k "prefetch or precast or adam or deferred or e2e or dp2 or grouped or gemm_group"
step $O/b64.txt timeout -k 10 300 python bench.py
step $O/b8.txt timeout -k 10 300 python bench.py --batch-per-gpu 8
echo done
