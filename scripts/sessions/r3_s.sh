cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r3s
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; if [ $rc -ne 0 ]; then echo "rc=$rc: $*" >> $O/rc.log; case $rc in 1|2) ;; *) exit $rc;; esac; fi; }
step $O/tests.log timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "attention"
[ -s $O/rc.log ] && exit 1
for i in 1 2; do
  step $O/b64_v1_$i.log env LJS_ATTN_VST=1 timeout -k 10 200 python bench.py
  step $O/b64_v0_$i.log env LJS_ATTN_VST=0 timeout -k 10 200 python bench.py
  step $O/b8_v1_$i.log env LJS_ATTN_VST=1 timeout -k 10 200 python bench.py --batch-per-gpu 8
  step $O/b8_v0_$i.log env LJS_ATTN_VST=0 timeout -k 10 200 python bench.py --batch-per-gpu 8
done
cd /tmp
for v in 1 0; do
  step $O/pb_$v.log env LJS_ATTN_VST=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/pb_$v -o run -- python3 $R/scripts/attn_one.py bwd 64 256 8 30
  step $O/pb8_$v.log env LJS_ATTN_VST=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/pb8_$v -o run -- python3 $R/scripts/attn_one.py bwd 8 256 8 30
done
for r in 16 108 116; do
  step $O/pf_r$r.log env LJS_ATTN_FWD_RES=$r timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/pf_r$r -o run -- python3 $R/scripts/attn_one.py fwd 64 256 8 30
done
echo done
