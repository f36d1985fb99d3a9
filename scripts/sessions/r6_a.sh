# round-6 session start: baseline of the inherited build on this round's box (driver shape x2, B=8,
# kernel trace of the B=64 step)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r6a
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
step $O/b64_1.txt timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5
step $O/b8_1.txt timeout -k 10 300 python bench.py --batch-per-gpu 8 --steps 20 --warmup 5
step $O/b64_2.txt timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5
cd /tmp
step $O/prof_b64.log timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof_b64 -o run -- python3 $R/bench.py --steps 20 --warmup 5
cd $R
python scripts/kstats.py $O/prof_b64/*/run_results.db --steps 87 > $O/b64_kernels.md 2>&1 || true
echo done
