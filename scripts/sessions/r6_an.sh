# round-6: the optimizer launch's next-input cast blocks with 4 chunks per thread (loads in flight
# together, a quarter of the blocks) vs 1: the bit-exact e2e test for both, then x3 interleaved
# steps at B=64 (driver shape) and B=8, and a B=8 / B=64 kernel trace of the new default
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r6an
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
step $O/tests.txt timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_e2e.py -k "input_cast_prefetch" -p no:cacheprovider
for rep in 1 2 3; do
  step $O/b64_u4_$rep.txt timeout -k 10 300 python scripts/bench_with.py adam_cast_u=4 -- --steps 20 --warmup 5
  step $O/b64_u1_$rep.txt timeout -k 10 300 python scripts/bench_with.py adam_cast_u=1 -- --steps 20 --warmup 5
  step $O/b8_u4_$rep.txt timeout -k 10 300 python scripts/bench_with.py adam_cast_u=4 -- --batch-per-gpu 8 --steps 20 --warmup 5
  step $O/b8_u1_$rep.txt timeout -k 10 300 python scripts/bench_with.py adam_cast_u=1 -- --batch-per-gpu 8 --steps 20 --warmup 5
done
for f in $O/b*_u*_*.txt; do echo "$(basename $f) $(grep -o '"ms_per_step": [0-9.]*' $f)"; done > $O/lines.txt
cd /tmp
step $O/prof_b8.log timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof_b8 -o run -- python3 $R/bench.py --batch-per-gpu 8 --steps 20 --warmup 5
step $O/prof_b64.log timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof_b64 -o run -- python3 $R/bench.py --steps 20 --warmup 5
cd $R
python scripts/kstats.py $O/prof_b8/run_results.db --steps 87 > $O/b8_kernels.md 2>&1
python scripts/kstats.py $O/prof_b64/run_results.db --steps 86 > $O/b64_kernels.md 2>&1
echo done
