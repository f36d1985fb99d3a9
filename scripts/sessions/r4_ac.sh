# automatic LDS-DMA K/V staging in the fused attention backward (<= 128 queries): attention tests,
# 2-D rehearsal / headline lines; aten trace of the 2-D MX-fp8 layer rehearsal's torch kernels
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r4ac
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then case $rc in 1|2) ;; *) exit $rc;; esac; fi; }
step $O/attn_tests.log timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "attention"
if grep -q " failed\|[0-9] error" $O/attn_tests.log; then echo "tests failed"; tail -40 $O/attn_tests.log; exit 1; fi
F4="WORLD_SIZE=4 RANK=0 LOCAL_RANK=0 LJS_DIST_BACKEND=fake MASTER_ADDR=127.0.0.1"
step $O/trace_2d_fp8.log env $F4 MASTER_PORT=29931 LJS_ATEN_TRACE=$O/aten_2d_fp8.txt timeout -k 10 300 python bench.py --gpus 4 --mesh 2d --model layer --fp8 --steps 2 --warmup 2 --min-warmup 0
for i in 1 2; do
step $O/f4_2d_$i.log env $F4 MASTER_PORT=2993$i timeout -k 10 200 python bench.py --gpus 4 --mesh 2d --steps 20 --warmup 5
step $O/drv_$i.log timeout -k 10 200 python bench.py --steps 20 --warmup 5
done
for f in $O/f4_*.log $O/drv*.log; do grep -h ms_per_step $f | python -c "
import sys,json
for l in sys.stdin:
    r=json.loads(l); print('$(basename $f)', r['ms_per_step'], r['value'])
" >> $O/summary.txt || true; done
echo done
