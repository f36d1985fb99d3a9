# final state: 64x64 bf16 GEMMs (the B=8 out-projection / dX) through the compile-time epilogue
# instances; full GPU suite + smoke; B=8 / B=64 A/B against LJS_GEMM_PLAIN=0; final tables
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r4x
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then case $rc in 1|2) ;; *) exit $rc;; esac; fi; }
step $O/gpu_tests.log timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/
if grep -q " failed\|[0-9] error" $O/gpu_tests.log; then echo "tests failed"; tail -40 $O/gpu_tests.log; exit 1; fi
step $O/smoke.log timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()"
for i in 1 2 3; do
step $O/b8_def_$i.log timeout -k 10 200 python bench.py --batch-per-gpu 8 --steps 20 --warmup 5
step $O/b8_gen_$i.log env LJS_GEMM_PLAIN=0 timeout -k 10 200 python bench.py --batch-per-gpu 8 --steps 20 --warmup 5
step $O/drv_$i.log timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5
step $O/drv_gen_$i.log env LJS_GEMM_PLAIN=0 timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5
done
step $O/layer_fp8.log timeout -k 10 200 python bench.py --model layer --fp8 --steps 20 --warmup 5
cd /tmp
step $O/prof_b64.log timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_b64 -o run -- python3 $R/bench.py --steps 16 --warmup 4
step $O/prof_b8.log timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_b8 -o run -- python3 $R/bench.py --batch-per-gpu 8 --steps 16 --warmup 4
cd $R
for p in prof_b64 prof_b8; do
  nn=$(grep -h ms_per_step $O/$p.log | python -c "import sys,json; r=json.loads(sys.stdin.readline()); print(r['warmup']+r['steps'])")
  python scripts/kstats.py $(ls $O/$p/*/run_results.db $O/$p/run_results.db 2>/dev/null | head -1) --steps $nn --title "$p" --out $O/$p.md || true
done
for f in $O/b8_*.log $O/drv_*.log $O/layer_*.log; do grep -h ms_per_step $f | python -c "
import sys,json
for l in sys.stdin:
    r=json.loads(l); print('$(basename $f)', r['ms_per_step'], r['value'])
" >> $O/summary.txt || true; done
echo done
