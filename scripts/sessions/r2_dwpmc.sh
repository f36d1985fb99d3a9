set -e
cd "$GRAFT_REPO_ROOT"
R=$PWD
mkdir -p gpurun_out/r2dw
timeout -k 10 120 python scripts/gemm_one.py dwslab:640:1536 1282 8 > gpurun_out/r2dw/t.log 2>&1
timeout -k 10 120 python scripts/gemm_one.py dwslab:2560:640 1282 5 >> gpurun_out/r2dw/t.log 2>&1
timeout -k 10 120 python scripts/gemm_one.py dwslab:640:2560 1282 5 >> gpurun_out/r2dw/t.log 2>&1
timeout -k 10 120 python scripts/gemm_one.py dwslab:512:640 1282 24 >> gpurun_out/r2dw/t.log 2>&1
timeout -k 10 120 python scripts/gemm_one.py dwslab:640:1536 12883 8 >> gpurun_out/r2dw/t.log 2>&1
timeout -k 10 120 python scripts/gemm_one.py dwslab:640:1536 12884 4 >> gpurun_out/r2dw/t.log 2>&1
timeout -k 10 120 python scripts/gemm_one.py dwslab:640:1536 1284 4 >> gpurun_out/r2dw/t.log 2>&1
cd /tmp && export TMPDIR=/tmp
run() {
  local name=$1; shift; local pass=$1; shift
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $pass --output-format csv -d "$R/gpurun_out/r2dw/$name" -- "$@" > "$R/gpurun_out/r2dw/$name.log" 2>&1
}
P1="SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"
P3="SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
run qkv_1 "$P1" python3 $R/scripts/gemm_one.py dwslab:640:1536 1282 8 20
run qkv_3 "$P3" python3 $R/scripts/gemm_one.py dwslab:640:1536 1282 8 20
run fwd_1 "$P1" python3 $R/scripts/gemm_one.py qkv 1282 1 20
run fwd_3 "$P3" python3 $R/scripts/gemm_one.py qkv 1282 1 20
cd "$R"
for d in gpurun_out/r2dw/*/; do python3 scripts/pmc_summary.py "$d**/*counter_collection.csv" > "${d%/}.txt" || true; done
