# last validation of the final tree: full GPU suite, smoke, default bench line
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r4ak
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then case $rc in 1|2) ;; *) exit $rc;; esac; fi; }
step $O/gpu_tests.log timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/
if grep -q " failed\|[0-9] error" $O/gpu_tests.log; then echo "tests failed"; tail -40 $O/gpu_tests.log; exit 1; fi
step $O/smoke.log timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()"
step $O/def.log timeout -k 10 300 python bench.py
tail -1 $O/gpu_tests.log; tail -1 $O/smoke.log; tail -1 $O/def.log
echo done
