cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r3ai
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; if [ $rc -ne 0 ]; then echo "rc=$rc: $*" >> $O/rc.log; case $rc in 1|2) ;; *) exit $rc;; esac; fi; }
step $O/tests.log timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "slab"
[ -s $O/rc.log ] && exit 1
for i in 1 2 3; do
  for v in 1 0; do
    step $O/b64_v${v}_$i.log env LJS_SLAB_VST=$v timeout -k 10 200 python bench.py
    step $O/b8_v${v}_$i.log env LJS_SLAB_VST=$v timeout -k 10 200 python bench.py --batch-per-gpu 8
  done
done
cd /tmp
for v in 1 0; do
  step $O/prof_b8_v$v.log env LJS_SLAB_VST=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_b8_v$v -o run -- python3 $R/bench.py --batch-per-gpu 8 --steps 16 --warmup 4
done
echo done
