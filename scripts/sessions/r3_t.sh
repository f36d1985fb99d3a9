cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r3t
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; if [ $rc -ne 0 ]; then echo "rc=$rc: $*" >> $O/rc.log; case $rc in 1|2) ;; *) exit $rc;; esac; fi; }
step $O/tests.log timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "attention"
[ -s $O/rc.log ] && exit 1
cd /tmp
for v in 1 2 0; do
  step $O/pb_$v.log env LJS_ATTN_VST=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/pb_$v -o run -- python3 $R/scripts/attn_one.py bwd 64 256 8 30
done
for v in 1 2 0; do
  step $O/prof_b64_$v.log env LJS_ATTN_VST=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_b64_$v -o run -- python3 $R/bench.py --steps 16 --warmup 4
done
echo done
