cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r3ak
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; if [ $rc -ne 0 ]; then echo "rc=$rc: $*" >> $O/rc.log; case $rc in 1|2) ;; *) exit $rc;; esac; fi; }
for i in 1 2 3; do
  step $O/drv_$i.log timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5
  step $O/def_$i.log timeout -k 10 200 python bench.py
  step $O/b8drv_$i.log timeout -k 10 200 python bench.py --batch-per-gpu 8 --steps 20 --warmup 5
done
step $O/rehearsal.log timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_rehearsal_gpu.py tests/test_bench_cpu.py
echo done
