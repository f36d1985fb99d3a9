# plain f32 split-K slab instance for the weight-gradient GEMMs (LJS_GEMM_PLAIN=0: general kernel);
# Adam: global (not flat) loads, double-buffered slab groups in the 32-row tile (LJS_ADAM_ROWS=32)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r4t
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then case $rc in 1|2) ;; *) exit $rc;; esac; fi; }
step $O/tests.log timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_gpu_e2e.py -k "gemm or slab or adam or optim or train"
if grep -q " failed\|[0-9] error" $O/tests.log; then echo "tests failed"; tail -30 $O/tests.log; exit 1; fi
step $O/tests_a32.log env LJS_ADAM_ROWS=32 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "adam and not mx"
if grep -q " failed\|[0-9] error" $O/tests_a32.log; then echo "tests failed"; tail -30 $O/tests_a32.log; exit 1; fi
for i in 1 2 3; do
step $O/gemm_plain_$i.log timeout -k 10 200 python scripts/gemm_ab.py dwqkv dwo
step $O/gemm_gen_$i.log env LJS_GEMM_PLAIN=0 timeout -k 10 200 python scripts/gemm_ab.py dwqkv dwo
done
for i in 1 2 3; do
step $O/b64_def_$i.log timeout -k 10 200 python bench.py --steps 20 --warmup 5
step $O/b64_a32_$i.log env LJS_ADAM_ROWS=32 timeout -k 10 200 python bench.py --steps 20 --warmup 5
step $O/b8_def_$i.log timeout -k 10 200 python bench.py --batch-per-gpu 8 --steps 20 --warmup 5
step $O/b8_a32_$i.log env LJS_ADAM_ROWS=32 timeout -k 10 200 python bench.py --batch-per-gpu 8 --steps 20 --warmup 5
done
cd /tmp
step $O/prof_b64.log timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_b64 -o run -- python3 $R/bench.py --steps 16 --warmup 4
step $O/prof_b64_a32.log env LJS_ADAM_ROWS=32 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_b64_a32 -o run -- python3 $R/bench.py --steps 16 --warmup 4
step $O/prof_b8.log timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_b8 -o run -- python3 $R/bench.py --batch-per-gpu 8 --steps 16 --warmup 4
step $O/prof_b8_a32.log env LJS_ADAM_ROWS=32 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_b8_a32 -o run -- python3 $R/bench.py --batch-per-gpu 8 --steps 16 --warmup 4
cd $R
for p in prof_b64 prof_b64_a32 prof_b8 prof_b8_a32; do
  n=$(grep -h ms_per_step $O/$p.log | python -c "import sys,json; r=json.loads(sys.stdin.readline()); print(r['warmup']+r['steps'])")
  python scripts/kstats.py $(ls $O/$p/*/run_results.db $O/$p/run_results.db 2>/dev/null | head -1) --steps $n --title "$p" --out $O/$p.md || true
done
for f in $O/b*.log; do grep -h ms_per_step $f | python -c "
import sys,json
for l in sys.stdin:
    r=json.loads(l); print('$(basename $f)', r['ms_per_step'])
" >> $O/summary.txt || true; done
echo done
