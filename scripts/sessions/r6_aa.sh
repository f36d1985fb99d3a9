# round-6: the fused projection + attention below one item per CU (B = 16: 128 items; B = 24: 192)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r6aa
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
for rep in 1 2 3; do
  for b in 16 24; do
    step $O/b${b}_on_$rep.txt timeout -k 10 300 python scripts/bench_with.py qkv_gate=1 -- --batch-per-gpu $b --steps 20 --warmup 5
    step $O/b${b}_off_$rep.txt timeout -k 10 300 python bench.py --batch-per-gpu $b --steps 20 --warmup 5
  done
done
for f in $O/b*_*.txt; do echo "$(basename $f) $(grep -o '"ms_per_step": [0-9.]*' $f)"; done > $O/lines.txt
echo done
