# round-6 final validation (after the capture-cut fix and the cast-transpose kernel): every GPU test, smoke(), driver-shape benches, a B=64 and a B=8 kernel trace
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r6al
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
step $O/tests.txt timeout -k 10 1100 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/
step $O/smoke.txt timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()"
step $O/b64_1.txt timeout -k 10 300 python bench.py --steps 20 --warmup 5
step $O/b64_2.txt timeout -k 10 300 python bench.py --steps 20 --warmup 5
step $O/b64_3.txt timeout -k 10 300 python bench.py --steps 20 --warmup 5
step $O/b8_1.txt timeout -k 10 300 python bench.py --batch-per-gpu 8 --steps 20 --warmup 5
step $O/def_1.txt timeout -k 10 300 python bench.py
step $O/l8_1.txt timeout -k 10 300 python bench.py --model layer --fp8 --steps 20 --warmup 5
for f in $O/b*_*.txt $O/def_*.txt $O/l8_*.txt; do echo "$(basename $f) $(grep -o '"ms_per_step": [0-9.]*' $f)"; done > $O/lines.txt
cd /tmp
step $O/prof_b64.log timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof_b64 -o run -- python3 $R/bench.py --steps 20 --warmup 5
step $O/prof_b8.log timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof_b8 -o run -- python3 $R/bench.py --batch-per-gpu 8 --steps 20 --warmup 5
cd $R
python scripts/kstats.py $O/prof_b64/run_results.db --steps 86 > $O/b64_kernels.md 2>&1
python scripts/kstats.py $O/prof_b8/run_results.db --steps 87 > $O/b8_kernels.md 2>&1
echo done
