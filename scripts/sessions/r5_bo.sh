# closing check: full GPU suite and smoke on the committed tree
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r5bo
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
step $O/gpu_tests.txt timeout -k 10 1000 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/
step $O/smoke.txt timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()"
step $O/b64_driver.txt timeout -k 10 300 python bench.py --steps 20 --warmup 5
echo done
