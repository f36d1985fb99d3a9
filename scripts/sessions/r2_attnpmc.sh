set -e
cd "$GRAFT_REPO_ROOT"
R=$PWD
mkdir -p gpurun_out/r2ap
cd /tmp && export TMPDIR=/tmp
run() {
  local name=$1; shift; local pass=$1; shift
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $pass --output-format csv -d "$R/gpurun_out/r2ap/$name" -- "$@" > "$R/gpurun_out/r2ap/$name.log" 2>&1
}
P1="SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"
P3="SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
P4="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM_RD SQ_INSTS_SMEM SQ_WAIT_INST_ANY SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_INSTS_VALU_TRANS_F32"
run bwd_1 "$P1" python3 $R/scripts/attn_one.py bwd 64 256 8 10
run bwd_3 "$P3" python3 $R/scripts/attn_one.py bwd 64 256 8 10
run bwd_4 "$P4" python3 $R/scripts/attn_one.py bwd 64 256 8 10
run fwd_1 "$P1" python3 $R/scripts/attn_one.py fwd 64 256 8 10
run fwd_3 "$P3" python3 $R/scripts/attn_one.py fwd 64 256 8 10
cd "$R"
for d in gpurun_out/r2ap/*/; do python3 scripts/pmc_summary.py "$d**/*counter_collection.csv" > "${d%/}.txt" || true; done
