# round-6: the split (pair32) attention backward at B = 64 vs the fused one (whose two rounds of
# blocks load in phase: profiles/r6t_attn_phases.txt)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r6w
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
for rep in 1 2 3; do
  step $O/b64_fused_$rep.txt timeout -k 10 300 python bench.py --steps 20 --warmup 5
  step $O/b64_split_$rep.txt timeout -k 10 300 python scripts/bench_with.py bwd_fused=0 -- --steps 20 --warmup 5
done
for f in $O/b*_*.txt; do echo "$(basename $f) $(grep -o '"ms_per_step": [0-9.]*' $f)"; done > $O/lines.txt
cd /tmp
step $O/prof_split.log timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof_split -o run -- python3 $R/scripts/bench_with.py bwd_fused=0 -- --steps 20 --warmup 5
cd $R
python scripts/kstats.py $O/prof_split/run_results.db --steps 86 > $O/split_kernels.md 2>&1
echo done
