set -e
cd "$GRAFT_REPO_ROOT"
scripts/pmc_gemm2.sh gpurun_out/pmc3 "qkv 1282 1" "dwqkv 1282 8" > gpurun_out/pmc3.log 2>&1
