# MX-fp8 GEMM f32-output instance (FIX 3; LJS_F8_FIX3=0 off) for the FF weight gradients; full GPU
# suite + smoke on the final state; fp8 layer A/B and table; headline lines
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r4z
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then case $rc in 1|2) ;; *) exit $rc;; esac; fi; }
step $O/gpu_tests.log timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/
if grep -q " failed\|[0-9] error" $O/gpu_tests.log; then echo "tests failed"; tail -40 $O/gpu_tests.log; exit 1; fi
step $O/smoke.log timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()"
for i in 1 2 3; do
step $O/l8_fix3_$i.log timeout -k 10 200 python bench.py --model layer --fp8 --steps 20 --warmup 5
step $O/l8_gen_$i.log env LJS_F8_FIX3=0 timeout -k 10 200 python bench.py --model layer --fp8 --steps 20 --warmup 5
step $O/drv_$i.log timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5
step $O/b8_$i.log timeout -k 10 200 python bench.py --batch-per-gpu 8 --steps 20 --warmup 5
done
cd /tmp
step $O/prof_l8.log timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_l8 -o run -- python3 $R/bench.py --model layer --fp8 --steps 16 --warmup 4
step $O/prof_l8_gen.log env LJS_F8_FIX3=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_l8_gen -o run -- python3 $R/bench.py --model layer --fp8 --steps 16 --warmup 4
cd $R
for p in prof_l8 prof_l8_gen; do
  nn=$(grep -h ms_per_step $O/$p.log | python -c "import sys,json; r=json.loads(sys.stdin.readline()); print(r['warmup']+r['steps'])")
  python scripts/kstats.py $(ls $O/$p/*/run_results.db $O/$p/run_results.db 2>/dev/null | head -1) --steps $nn --title "$p" --out $O/$p.md || true
done
for f in $O/l8_*.log $O/drv_*.log $O/b8_*.log; do grep -h ms_per_step $f | python -c "
import sys,json
for l in sys.stdin:
    r=json.loads(l); print('$(basename $f)', r['ms_per_step'], r['value'])
" >> $O/summary.txt || true; done
echo done
