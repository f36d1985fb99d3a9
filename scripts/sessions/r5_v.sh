# round-5 checkpoint validation of the committed tree: the full GPU suite, smoke(), driver-shaped
# bench lines (B=64 x3, B=8 x2, no-flag), fp8 / bf16 layer lines, B=64 / B=8 kernel tables
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r5v
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
step $O/gpu_tests.txt timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/
step $O/smoke.txt timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
for rep in 1 2 3; do
  step $O/drv_b64_$rep.txt timeout -k 10 300 python bench.py --steps 20 --warmup 5
done
for rep in 1 2; do
  step $O/drv_b8_$rep.txt timeout -k 10 300 python bench.py --steps 20 --warmup 5 --batch-per-gpu 8
done
step $O/noflag.txt timeout -k 10 300 python bench.py
step $O/layer_fp8.txt timeout -k 10 300 python bench.py --model layer --fp8
step $O/layer_bf16.txt timeout -k 10 300 python bench.py --model layer
cd /tmp
step $O/prof_b64.log timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_b64 -o run -- python3 $R/bench.py --steps 16 --warmup 4
step $O/prof_b8.log timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_b8 -o run -- python3 $R/bench.py --batch-per-gpu 8 --steps 16 --warmup 4
cd $R
for p in b64 b8; do
  nn=$(grep -h ms_per_step $O/prof_$p.log | python -c "import sys,json; r=json.loads(sys.stdin.readline()); print(r['warmup']+r['steps'])")
  python scripts/kstats.py $(ls $O/prof_$p/*/run_results.db $O/prof_$p/run_results.db 2>/dev/null | head -1) --steps $nn --title "r5v $p" --out $O/prof_$p.md > /dev/null 2>&1 || true
done
echo done
