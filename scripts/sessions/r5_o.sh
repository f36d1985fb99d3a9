# Adam per-tensor tile height (32-row tiles for >= 16-slab gradients; LJS_ADAM_SPLIT_S=0 off) and
# the count-increment form: GPU tests, probe, then same-box bench A/B at B=64 and B=8, step tables
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r5o
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
step $O/tests.txt timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu -k "adam or optim or step or train" tests/
step $O/probe_split16.txt timeout -k 10 120 python scripts/adam_probe.py
LJS_ADAM_SPLIT_S=0 step $O/probe_split0.txt timeout -k 10 120 python scripts/adam_probe.py
for rep in 1 2; do
  for b in 64 8; do
    step $O/bench_b${b}_default_$rep.txt timeout -k 10 300 python bench.py --batch-per-gpu $b
    LJS_ADAM_SPLIT_S=0 step $O/bench_b${b}_split0_$rep.txt timeout -k 10 300 python bench.py --batch-per-gpu $b
    LJS_ADAM_STEP_INC=ticket step $O/bench_b${b}_ticket_$rep.txt timeout -k 10 300 python bench.py --batch-per-gpu $b
  done
done
cd /tmp
step $O/prof_b64.log timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_b64 -o run -- python3 $R/bench.py --steps 16 --warmup 4
cd $R
nn=$(grep -h ms_per_step $O/prof_b64.log | python -c "import sys,json; r=json.loads(sys.stdin.readline()); print(r['warmup']+r['steps'])")
python scripts/kstats.py $(ls $O/prof_b64/*/run_results.db $O/prof_b64/run_results.db 2>/dev/null | head -1) --steps $nn --title b64 --out $O/prof_b64.md > /dev/null 2>&1 || true
echo done
