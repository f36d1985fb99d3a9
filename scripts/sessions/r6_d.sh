# round-6: after the variant pruning -- the kernel / epilogue / e2e GPU tests, the driver-shape
# bench, then per-kernel memory-side bytes + instruction mix of the headline step (roofline
# table) and fresh kernel traces of the MX-fp8 layer and of B=8
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r6d
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
step $O/tests.txt timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_epilogue_gpu.py tests/test_gpu_e2e.py
step $O/b64.txt timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5
step $O/b8.txt timeout -k 10 300 python bench.py --batch-per-gpu 8 --steps 20 --warmup 5
cd /tmp
step $O/pmc_b64.log timeout -s KILL 150 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU --output-format csv -d $O/pmc_b64 -- python3 $R/bench.py --steps 4 --warmup 2 --min-warmup 0 --graph-steps 1
step $O/prof_fp8.log timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof_fp8 -o run -- python3 $R/bench.py --model layer --fp8 --steps 20 --warmup 5
step $O/prof_b8.log timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof_b8 -o run -- python3 $R/bench.py --batch-per-gpu 8 --steps 20 --warmup 5
cd $R
python scripts/pmc_summary.py "$O/pmc_b64/**/*counter_collection.csv" > $O/pmc_b64.txt 2>&1
python scripts/kstats.py $O/prof_fp8/run_results.db --steps 86 > $O/fp8_kernels.md 2>&1
python scripts/kstats.py $O/prof_b8/run_results.db --steps 87 > $O/b8_kernels.md 2>&1
echo done
