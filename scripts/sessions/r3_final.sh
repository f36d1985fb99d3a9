cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r3final3
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; if [ $rc -ne 0 ]; then echo "rc=$rc: $*" >> $O/rc.log; case $rc in 1|2) ;; *) exit $rc;; esac; fi; }
step $O/gpu_tests.log timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/
step $O/smoke.log timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step $O/bench_default.log timeout -k 10 300 python bench.py
step $O/bench_driver.log timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5
step $O/b8.log timeout -k 10 300 python bench.py --batch-per-gpu 8
step $O/l8.log timeout -k 10 300 python bench.py --model layer --fp8
echo done
