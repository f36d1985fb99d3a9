# round-6: the lowered fused-projection gate (>= one item per two CUs) at B = 12 (96 items, off by
# the gate; forced on for the A/B), then the driver's multi-rank launch form over gloo (r6_ab.sh)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$PWD/gpurun_out/r6ac
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
for rep in 1 2 3; do
  step $O/b12_on_$rep.txt timeout -k 10 300 python scripts/bench_with.py qkv_gate=1 -- --batch-per-gpu 12 --steps 20 --warmup 5
  step $O/b12_off_$rep.txt timeout -k 10 300 python bench.py --batch-per-gpu 12 --steps 20 --warmup 5
done
step $O/b16_default.txt timeout -k 10 300 python bench.py --batch-per-gpu 16 --steps 20 --warmup 5
for f in $O/b*.txt; do echo "$(basename $f) $(grep -o '"ms_per_step": [0-9.]*' $f)"; done > $O/lines.txt
bash scripts/sessions/r6_ab.sh
