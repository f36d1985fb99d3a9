cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r3z
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; if [ $rc -ne 0 ]; then echo "rc=$rc: $*" >> $O/rc.log; case $rc in 1|2) ;; *) exit $rc;; esac; fi; }
step $O/gpu_tests.log timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/
step $O/smoke.log timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
for i in 1 2; do
  step $O/b64_$i.log timeout -k 10 200 python bench.py
  step $O/b8_$i.log timeout -k 10 200 python bench.py --batch-per-gpu 8
done
step $O/mse.log timeout -k 10 200 python bench.py --loss mse
step $O/long.log timeout -k 10 200 python bench.py --seq 4096 --batch-per-gpu 4
step $O/l16.log timeout -k 10 200 python bench.py --model layer
cd /tmp
step $O/prof_b64.log timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_b64 -o run -- python3 $R/bench.py --steps 24 --warmup 6
step $O/prof_b8.log timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_b8 -o run -- python3 $R/bench.py --batch-per-gpu 8 --steps 24 --warmup 6
echo done
