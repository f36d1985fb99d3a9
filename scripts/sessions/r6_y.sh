# round-6: per-kernel memory-side bytes + instruction mix of the final B=64 step (roofline table)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r6y
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
cd /tmp
step $O/pmc_b64.log timeout -s KILL 150 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU --output-format csv -d $O/pmc_b64 -- python3 $R/bench.py --steps 4 --warmup 2 --min-warmup 0 --graph-steps 1
step $O/pmc2_b64.log timeout -s KILL 150 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_INSTS_SALU --output-format csv -d $O/pmc2_b64 -- python3 $R/bench.py --steps 4 --warmup 2 --min-warmup 0 --graph-steps 1
cd $R
python scripts/pmc_summary.py "$O/pmc_b64/**/*counter_collection.csv" > $O/pmc_b64.txt 2>&1
python scripts/pmc_summary.py "$O/pmc2_b64/**/*counter_collection.csv" > $O/pmc2_b64.txt 2>&1
echo done
