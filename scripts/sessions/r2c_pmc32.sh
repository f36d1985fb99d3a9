set -e
cd "$GRAFT_REPO_ROOT"
R=$PWD
mkdir -p gpurun_out/r2c_pmc32
cd /tmp && export TMPDIR=/tmp
for v in 0 1; do
timeout -s KILL 90 env LJS_ATTN_DKV32=$v LJS_ATTN_DQ32=$v rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT \
  --output-format csv -d $R/gpurun_out/r2c_pmc32/a$v -- python3 $R/scripts/attn_one.py bwd 4 4096 8 6 > $R/gpurun_out/r2c_pmc32/a$v.log 2>&1
timeout -s KILL 90 env LJS_ATTN_DKV32=$v LJS_ATTN_DQ32=$v rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC \
  --output-format csv -d $R/gpurun_out/r2c_pmc32/b$v -- python3 $R/scripts/attn_one.py bwd 4 4096 8 6 > $R/gpurun_out/r2c_pmc32/b$v.log 2>&1
done
