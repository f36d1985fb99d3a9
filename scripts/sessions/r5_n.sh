# Adam count increment: separate one-lane launch (default) vs the in-kernel ticket forms
# (LJS_ADAM_STEP_INC=ticket, LJS_ADAM_EARLY_TICKET=0 end-of-block two-level, 1 early two-level,
# 2 early one word) in scripts/adam_probe.py; then the B=64 / B=8 step tables with the default
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r5n
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
step $O/tests.txt timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu -k "adam or optim or step or train" tests/
step $O/inc_kernel.txt timeout -k 10 120 python scripts/adam_probe.py
for e in 0 1 2; do
  LJS_ADAM_STEP_INC=ticket LJS_ADAM_EARLY_TICKET=$e step $O/inc_ticket$e.txt timeout -k 10 120 python scripts/adam_probe.py
done
cd /tmp
for cfg in "b64 64" "b8 8"; do
  set -- $cfg
  step $O/prof_$1.log timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$1 -o run -- python3 $R/bench.py --batch-per-gpu $2 --steps 16 --warmup 4
done
cd $R
for p in b64 b8; do
  nn=$(grep -h ms_per_step $O/prof_$p.log | python -c "import sys,json; r=json.loads(sys.stdin.readline()); print(r['warmup']+r['steps'])")
  python scripts/kstats.py $(ls $O/prof_$p/*/run_results.db $O/prof_$p/run_results.db 2>/dev/null | head -1) --steps $nn --title "$p" --out $O/prof_$p.md > /dev/null 2>&1 || true
done
for b in 64 8; do
  step $O/bench_b$b.txt timeout -k 10 300 python bench.py --batch-per-gpu $b
done
echo done
