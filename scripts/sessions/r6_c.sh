# round-6: per-kernel memory-side bytes + instruction mix of the headline step (roofline table),
# fresh kernel traces of the MX-fp8 layer and of B=8 on the current build
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r6c
mkdir -p $O
cd /tmp
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU --output-format csv -d $O/pmc_b64 -- python3 $R/bench.py --steps 4 --warmup 2 --min-warmup 0 --graph-steps 1 > $O/pmc_b64.log 2>&1 || exit 3
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU --output-format csv -d $O/pmc_b8 -- python3 $R/bench.py --batch-per-gpu 8 --steps 4 --warmup 2 --min-warmup 0 --graph-steps 1 > $O/pmc_b8.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof_fp8 -o run -- python3 $R/bench.py --model layer --fp8 --steps 20 --warmup 5 > $O/prof_fp8.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof_b8 -o run -- python3 $R/bench.py --batch-per-gpu 8 --steps 20 --warmup 5 > $O/prof_b8.log 2>&1 || exit 3
cd $R
python scripts/pmc_summary.py "$O/pmc_b64/**/*counter_collection.csv" > $O/pmc_b64.txt 2>&1
python scripts/pmc_summary.py "$O/pmc_b8/**/*counter_collection.csv" > $O/pmc_b8.txt 2>&1
python scripts/kstats.py $O/prof_fp8/run_results.db --steps 86 > $O/fp8_kernels.md 2>&1
python scripts/kstats.py $O/prof_b8/run_results.db --steps 87 > $O/b8_kernels.md 2>&1
echo done
