cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d gpurun_out/pmc_attn1 -o run --output-format csv -- python scripts/attn_one.py fwd > gpurun_out/pmc_attn1.log 2>&1 || echo "pass1 rc=$?"
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum TA_BUSY_avr TCP_TOTAL_CACHE_ACCESSES_sum SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM SQ_LDS_IDX_ACTIVE -d gpurun_out/pmc_attn2 -o run --output-format csv -- python scripts/attn_one.py fwd > gpurun_out/pmc_attn2.log 2>&1 || echo "pass2 rc=$?"
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_SALU SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM GRBM_GUI_ACTIVE -d gpurun_out/pmc_attn3 -o run --output-format csv -- python scripts/attn_one.py fwd > gpurun_out/pmc_attn3.log 2>&1 || echo "pass3 rc=$?"
