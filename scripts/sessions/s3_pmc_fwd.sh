cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
i=0
for pass in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
            "SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU" \
            "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $pass --output-format csv -d gpurun_out/s3_pmcf/p$i -- python scripts/attn_one.py fwd > gpurun_out/s3_pmcf_p$i.log 2>&1 || { echo "pass $i rc=$?"; exit 1; }
done
for i in 1 2 3; do python scripts/pmc_summary.py "gpurun_out/s3_pmcf/p$i/**/*counter_collection.csv" | grep -A12 "attn_fwd" ; done > gpurun_out/s3_pmcf_summary.txt
