set -e
cd "$GRAFT_REPO_ROOT"
R=$PWD
mkdir -p gpurun_out/r2pmc
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT \
  --output-format csv -d $R/gpurun_out/r2pmc/a1 -- python3 $R/scripts/attn_one.py bwd 64 256 8 20 > $R/gpurun_out/r2pmc/a1.log 2>&1
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC \
  --output-format csv -d $R/gpurun_out/r2pmc/a2 -- python3 $R/scripts/attn_one.py bwd 64 256 8 20 > $R/gpurun_out/r2pmc/a2.log 2>&1
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT \
  --output-format csv -d $R/gpurun_out/r2pmc/f1 -- python3 $R/scripts/attn_one.py fwd 64 256 8 20 > $R/gpurun_out/r2pmc/f1.log 2>&1
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC \
  --output-format csv -d $R/gpurun_out/r2pmc/f2 -- python3 $R/scripts/attn_one.py fwd 64 256 8 20 > $R/gpurun_out/r2pmc/f2.log 2>&1
