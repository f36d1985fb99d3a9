set -e
cd "$GRAFT_REPO_ROOT"
R=$PWD
mkdir -p gpurun_out/r2dw3
o=gpurun_out/r2dw3/t.log
: > $o
for cfg in "dwslab:640:1536 1282 8" "dwkc:640:1536 1282 8" "dwall_slabs 1282 8" "dwslab:640:1536 1284 4" "dwslab:640:1536 12884 4" "dwslab:640:1536 1282 4"; do
  timeout -k 10 120 python scripts/gemm_one.py $cfg 50 2>&1 | grep -v amdgpu.ids >> $o
done
cd /tmp && export TMPDIR=/tmp
run() {
  local name=$1; shift; local pass=$1; shift
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $pass --output-format csv -d "$R/gpurun_out/r2dw3/$name" -- "$@" > "$R/gpurun_out/r2dw3/$name.log" 2>&1
}
P2="TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"
P4="TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TA_BUSY_avr TCC_EA0_RDREQ_DRAM_sum"
run dw_2 "$P2" python3 $R/scripts/gemm_one.py dwslab:640:1536 1282 8 20
run dw_4 "$P4" python3 $R/scripts/gemm_one.py dwslab:640:1536 1282 8 20
run kc_4 "$P4" python3 $R/scripts/gemm_one.py dwkc:640:1536 1282 8 20
run fwd_2 "$P2" python3 $R/scripts/gemm_one.py qkv 1282 1 20
run fwd_4 "$P4" python3 $R/scripts/gemm_one.py qkv 1282 1 20
cd "$R"
for d in gpurun_out/r2dw3/*/; do python3 scripts/pmc_summary.py "$d**/*counter_collection.csv" > "${d%/}.txt" || true; done
