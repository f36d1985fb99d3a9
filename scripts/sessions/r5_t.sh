# input-cast prefetch (ops/linear.prefetch_next_input): graph tests, then same-box bench A/B
# (LJS_PRECAST=0 / 1) at B=64 and B=8, and a B=64 kernel trace with it on
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r5t
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
step $O/tests.txt timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu -k "jit_graph or capture" tests/test_gpu_e2e.py tests/test_multi_gpu_capture_gpu.py
for rep in 1 2; do
  for b in 64 8; do
    LJS_PRECAST=0 step $O/b${b}_off_$rep.txt timeout -k 10 300 python bench.py --batch-per-gpu $b
    step $O/b${b}_on_$rep.txt timeout -k 10 300 python bench.py --batch-per-gpu $b
  done
done
cd /tmp
step $O/prof_b64.log timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_b64 -o run -- python3 $R/bench.py --steps 16 --warmup 4
cd $R
nn=$(grep -h ms_per_step $O/prof_b64.log | python -c "import sys,json; r=json.loads(sys.stdin.readline()); print(r['warmup']+r['steps'])")
python scripts/kstats.py $(ls $O/prof_b64/*/run_results.db $O/prof_b64/run_results.db 2>/dev/null | head -1) --steps $nn --title b64_precast --out $O/prof_b64.md > /dev/null 2>&1 || true
echo done
