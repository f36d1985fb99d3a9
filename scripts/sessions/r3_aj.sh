cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r3aj
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; if [ $rc -ne 0 ]; then echo "rc=$rc: $*" >> $O/rc.log; case $rc in 1|2) ;; *) exit $rc;; esac; fi; }
step $O/tests0.log env LJS_ATTN_BWD_KV_DMA=0 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "attention"
[ -s $O/rc.log ] && exit 1
for i in 1 2 3; do
  for v in 1 0; do
    step $O/b64_kv${v}_$i.log env LJS_ATTN_BWD_KV_DMA=$v timeout -k 10 200 python bench.py
  done
done
cd /tmp
for v in 1 0; do
  step $O/pb_$v.log env LJS_ATTN_BWD_KV_DMA=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/pb_$v -o run -- python3 $R/scripts/attn_one.py bwd 64 256 8 30
done
echo done
