# round-6: swap01 (x -> seq-major bf16) with 4 chunks per thread: its tests, the fake-4 2-D step
# (x2, interleaved with dp) and the 2-D kernel trace
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r6ak
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
step $O/tests.txt timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "swap01 or seq_major or elementwise" -p no:cacheprovider
export WORLD_SIZE=4 RANK=0 LOCAL_RANK=0 LJS_DIST_BACKEND=fake MASTER_ADDR=127.0.0.1 MASTER_PORT=29919
step $O/b2d_1.txt timeout -k 10 300 python bench.py --gpus 4 --mesh 2d --secondary off --steps 20 --warmup 5
step $O/bdp_1.txt timeout -k 10 300 python bench.py --gpus 4 --secondary off --steps 20 --warmup 5
step $O/b2d_2.txt timeout -k 10 300 python bench.py --gpus 4 --mesh 2d --secondary off --steps 20 --warmup 5
step $O/bdp_2.txt timeout -k 10 300 python bench.py --gpus 4 --secondary off --steps 20 --warmup 5
cd /tmp
step $O/prof_2d.log timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof_2d -o run -- python3 $R/bench.py --gpus 4 --mesh 2d --secondary off --steps 20 --warmup 5
cd $R
python scripts/kstats.py $O/prof_2d/run_results.db --steps 86 > $O/k2d.md 2>&1
for f in $O/b2d_?.txt $O/bdp_?.txt; do echo "$(basename $f) $(grep -o '"ms_per_step": [0-9.]*' $f)"; done > $O/lines.txt
echo done
