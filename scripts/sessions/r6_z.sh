# round-6: the fused projection + attention at one item per CU (B = 32) and at B = 16 (gated off)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r6z
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
for rep in 1 2 3; do
  step $O/b32_on_$rep.txt timeout -k 10 300 python bench.py --batch-per-gpu 32 --steps 20 --warmup 5
  step $O/b32_off_$rep.txt timeout -k 10 300 env LJS_QKV_ATTN=0 python bench.py --batch-per-gpu 32 --steps 20 --warmup 5
done
for f in $O/b*_*.txt; do echo "$(basename $f) $(grep -o '"ms_per_step": [0-9.]*' $f)"; done > $O/lines.txt
echo done
