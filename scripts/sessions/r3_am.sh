cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r3am
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; if [ $rc -ne 0 ]; then echo "rc=$rc: $*" >> $O/rc.log; case $rc in 1|2) ;; *) exit $rc;; esac; fi; }
for i in 1 2; do
  step $O/drv_$i.log timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5
  step $O/b8drv_$i.log timeout -k 10 200 python bench.py --batch-per-gpu 8 --steps 20 --warmup 5
done
step $O/def.log timeout -k 10 200 python bench.py
step $O/rehearsal.log timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_rehearsal_gpu.py tests/test_failure_detection.py
step $O/smoke.log timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
echo done
