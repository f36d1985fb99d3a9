cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r3y
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; if [ $rc -ne 0 ]; then echo "rc=$rc: $*" >> $O/rc.log; case $rc in 1|2) ;; *) exit $rc;; esac; fi; }
step $O/tests.log timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "fp8 or mx"
[ -s $O/rc.log ] && exit 1
step $O/one_down.log timeout -k 10 120 python scripts/fp8_one.py 640 2560 256160 30 res
step $O/one_dx.log timeout -k 10 120 python scripts/fp8_one.py 640 2560 256160 30
for i in 1 2; do
  step $O/l8_$i.log timeout -k 10 200 python bench.py --model layer --fp8
done
cd /tmp
step $O/prof_l8.log timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_l8 -o run -- python3 $R/bench.py --model layer --fp8 --steps 16 --warmup 4
echo done
