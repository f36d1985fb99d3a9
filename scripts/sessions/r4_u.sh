# fused attention backward: the common case's sweep as its own kernel instance (SW 1: 236 VGPRs,
# no spills, vs 256 + 7 VGPR / 32 SGPR spills with all four sweeps; LJS_ATTN_BWD_SW=0 off)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r4u
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then case $rc in 1|2) ;; *) exit $rc;; esac; fi; }
step $O/tests.log timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "attn or attention"
if grep -q " failed\|[0-9] error" $O/tests.log; then echo "tests failed"; tail -30 $O/tests.log; exit 1; fi
for i in 1 2 3; do
step $O/at_sw1_$i.log timeout -k 10 200 python scripts/attn_time.py
step $O/at_sw0_$i.log env LJS_ATTN_BWD_SW=0 timeout -k 10 200 python scripts/attn_time.py
done
for i in 1 2 3; do
step $O/b64_sw1_$i.log timeout -k 10 200 python bench.py --steps 20 --warmup 5
step $O/b64_sw0_$i.log env LJS_ATTN_BWD_SW=0 timeout -k 10 200 python bench.py --steps 20 --warmup 5
done
step $O/layer_fp8.log timeout -k 10 200 python bench.py --model layer --fp8 --steps 20 --warmup 5
step $O/layer_bf16.log timeout -k 10 200 python bench.py --model layer --steps 20 --warmup 5
cd /tmp
step $O/prof_b64.log timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_b64 -o run -- python3 $R/bench.py --steps 16 --warmup 4
step $O/prof_l8.log timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_l8 -o run -- python3 $R/bench.py --model layer --fp8 --steps 16 --warmup 4
cd $R
for p in prof_b64 prof_l8; do
  n=$(grep -h ms_per_step $O/$p.log | python -c "import sys,json; r=json.loads(sys.stdin.readline()); print(r['warmup']+r['steps'])")
  python scripts/kstats.py $(ls $O/$p/*/run_results.db $O/$p/run_results.db 2>/dev/null | head -1) --steps $n --title "$p" --out $O/$p.md || true
done
for f in $O/b*.log $O/l*.log; do grep -h ms_per_step $f | python -c "
import sys,json
for l in sys.stdin:
    r=json.loads(l); print('$(basename $f)', r['ms_per_step'])
" >> $O/summary.txt || true; done
echo done
