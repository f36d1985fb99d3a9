# round-6 closing check of the final tree (rebuilt library): every GPU test and smoke(), one driver-shape bench
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$PWD/gpurun_out/r6at
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
step $O/tests.txt timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/
step $O/smoke.txt timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()"
step $O/b64.txt timeout -k 10 300 python bench.py --steps 20 --warmup 5
echo done
