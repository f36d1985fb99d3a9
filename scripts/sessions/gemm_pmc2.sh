set -e
cd "$GRAFT_REPO_ROOT"
scripts/pmc_gemm.sh gpurun_out/pmcg2 "qkv 2561 1" "qkv 1282 1" > gpurun_out/pmc2.log 2>&1
