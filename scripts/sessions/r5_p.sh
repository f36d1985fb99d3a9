# L2 hit rate / memory-side reads per kernel (TCC counters): the headline step (one step per graph)
# and the weight-gradient / QKV GEMMs in isolation (scripts/gemm_cases.py)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r5p
mkdir -p $O
cd /tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum --output-format csv -d $O/pmc_step -- python3 $R/bench.py --steps 4 --warmup 2 --min-warmup 0 --graph-steps 1 > $O/pmc_step.log 2>&1 || exit 3
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum --output-format csv -d $O/pmc_iso -- python3 $R/scripts/gemm_cases.py dwqkv dwo qkv > $O/pmc_iso.log 2>&1 || exit 3
cd $R
python scripts/pmc_summary.py "$O/pmc_step/**/*counter_collection.csv" > $O/pmc_step.txt 2>&1
python scripts/pmc_summary.py "$O/pmc_iso/**/*counter_collection.csv" > $O/pmc_iso.txt 2>&1
echo done
