# (r5bd: final-build re-run of r5_j.sh) PMC passes over the headline step (B=64, one step per graph): per-kernel MFMA busy, VALU / LDS
# per MFMA, wait breakdown, LDS bank conflicts -- for the current build (lean GEMMs, 256x192 QKV)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r5bd
mkdir -p $O
cd /tmp
n=0
for pass in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
            "SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE" \
            "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM"; do
  n=$((n+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $pass --output-format csv -d $O/pmc_$n -- python3 $R/bench.py --steps 4 --warmup 2 --min-warmup 0 --graph-steps 1 > $O/pmc_$n.log 2>&1 || exit 3
done
cd $R
for n in 1 2 3; do python scripts/pmc_summary.py "$O/pmc_$n/**/*counter_collection.csv" > $O/pmc_$n.txt 2>&1 || true; done
echo done
# kernel traces of the final build at B=64 and B=8 (default step count)
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof_b64 -o run -- python3 $R/bench.py --steps 20 --warmup 5 > $O/prof_b64.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof_b8 -o run -- python3 $R/bench.py --batch-per-gpu 8 --steps 20 --warmup 5 > $O/prof_b8.log 2>&1 || exit 3
echo done2
