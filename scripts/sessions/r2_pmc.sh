set -e
cd "$GRAFT_REPO_ROOT"
R=$PWD
mkdir -p gpurun_out/r2p
cd /tmp && export TMPDIR=/tmp
run() {  # name pass cmd...
  local name=$1; shift; local pass=$1; shift
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $pass --output-format csv -d "$R/gpurun_out/r2p/$name" -- "$@" > "$R/gpurun_out/r2p/$name.log" 2>&1
}
P1="SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"
P2="TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"
run f8_2560_a "$P1" python3 $R/scripts/fp8_one.py 2560 640 2563
run f8_2560_b "$P2" python3 $R/scripts/fp8_one.py 2560 640 2563
run f8_640_a "$P1" python3 $R/scripts/fp8_one.py 640 2560 1282
run f8_640_b "$P2" python3 $R/scripts/fp8_one.py 640 2560 1282
run bf_qkv_a "$P1" python3 $R/scripts/gemm_one.py qkv 2561 1 20
run bf_qkv_b "$P2" python3 $R/scripts/gemm_one.py qkv 2561 1 20
run f8_2560q_a "$P1" python3 $R/scripts/fp8_one.py 2560 640 2563 20 qout
cd "$R"
for d in gpurun_out/r2p/*/; do python3 scripts/pmc_summary.py "$d**/*counter_collection.csv" > "${d%/}.txt" || true; done
