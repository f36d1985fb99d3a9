# final-build 2-D rehearsal kernel tables (bf16 and MX-fp8 layer, 4 fake ranks, rank 0) and the
# B=8 A/B of the out-projection bias+sum GEMM instance (LJS_GEMM_BSUM=0 off); fused attention
# backward with K / V by LDS-DMA (new one-sweep instance) A/B in the 2-D rehearsal and the headline
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r4ab
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then case $rc in 1|2) ;; *) exit $rc;; esac; fi; }
step $O/attn_tests.log timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "attention"
if grep -q " failed\|[0-9] error" $O/attn_tests.log; then echo "tests failed"; tail -40 $O/attn_tests.log; exit 1; fi
F4="WORLD_SIZE=4 RANK=0 LOCAL_RANK=0 LJS_DIST_BACKEND=fake MASTER_ADDR=127.0.0.1"
for i in 1 2 3; do
step $O/f4_2d_$i.log env $F4 MASTER_PORT=2991$i timeout -k 10 200 python bench.py --gpus 4 --mesh 2d --steps 20 --warmup 5
step $O/f4_2d_kvdma_$i.log env $F4 MASTER_PORT=2992$i LJS_ATTN_BWD_KV_DMA=1 timeout -k 10 200 python bench.py --gpus 4 --mesh 2d --steps 20 --warmup 5
step $O/drv_$i.log timeout -k 10 200 python bench.py --steps 20 --warmup 5
step $O/drv_kvdma_$i.log env LJS_ATTN_BWD_KV_DMA=1 timeout -k 10 200 python bench.py --steps 20 --warmup 5
done
for i in 1 2 3; do
step $O/b8_$i.log timeout -k 10 200 python bench.py --batch-per-gpu 8 --steps 20 --warmup 5
step $O/b8_nobsum_$i.log env LJS_GEMM_BSUM=0 timeout -k 10 200 python bench.py --batch-per-gpu 8 --steps 20 --warmup 5
done
cd /tmp
export WORLD_SIZE=4 RANK=0 LOCAL_RANK=0 LJS_DIST_BACKEND=fake MASTER_ADDR=127.0.0.1
step $O/prof_2d_kvdma.log env MASTER_PORT=29914 LJS_ATTN_BWD_KV_DMA=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_2d_kvdma -o run -- python3 $R/bench.py --gpus 4 --mesh 2d --steps 16 --warmup 4
step $O/prof_2d.log env MASTER_PORT=29911 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_2d -o run -- python3 $R/bench.py --gpus 4 --mesh 2d --steps 16 --warmup 4
step $O/prof_dp.log env MASTER_PORT=29912 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_dp -o run -- python3 $R/bench.py --gpus 4 --mesh dp --steps 16 --warmup 4
step $O/prof_2d_fp8.log env MASTER_PORT=29913 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_2d_fp8 -o run -- python3 $R/bench.py --gpus 4 --mesh 2d --model layer --fp8 --steps 16 --warmup 4
cd $R
for p in prof_2d prof_2d_kvdma prof_dp prof_2d_fp8; do
  nn=$(grep -h ms_per_step $O/$p.log | python -c "import sys,json; r=json.loads(sys.stdin.readline()); print(r['warmup']+r['steps'])")
  python scripts/kstats.py $(ls $O/$p/*/run_results.db $O/$p/run_results.db 2>/dev/null | head -1) --steps $nn --title "$p" --out $O/$p.md || true
done
for f in $O/f4_*.log $O/drv*.log $O/b8*.log $O/prof_*.log; do grep -h ms_per_step $f | python -c "
import sys,json
for l in sys.stdin:
    r=json.loads(l); print('$(basename $f)', r['ms_per_step'], r['value'])
" >> $O/summary.txt || true; done
echo done
