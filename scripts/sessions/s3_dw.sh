set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for cfg in "dwall 1282 8" "dwall 1282 4" "dwall_slabs 1282 8" "dwall_kc 1282 8" "dwall_kc 2561 1" "dwqkv 1282 8" "dwo 1282 16" "dwo_slabs 1282 16"; do
  timeout -k 10 60 python scripts/gemm_one.py $cfg >> gpurun_out/s3_dw_times.log 2>&1
done
timeout -k 10 600 bash scripts/pmc_gemm2.sh gpurun_out/s3_pmc "dwqkv 1282 8" "qkv 2561 1" > gpurun_out/s3_pmc.log 2>&1
