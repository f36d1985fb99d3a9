cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r3p
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; if [ $rc -ne 0 ]; then echo "rc=$rc: $*" >> $O/rc.log; case $rc in 1|2) ;; *) exit $rc;; esac; fi; }
step $O/tests.log timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "fp8 or colsum or rows_sum"
for i in 1 2; do
  step $O/l8_on_$i.log timeout -k 10 200 python bench.py --model layer --fp8
  step $O/l8_off_$i.log env LJS_F8_FUSED_COLSUM=0 timeout -k 10 200 python bench.py --model layer --fp8
done
cd /tmp
step $O/prof_layer8.log timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_layer8 -o run -- python3 $R/bench.py --model layer --fp8 --steps 24 --warmup 6
echo done
