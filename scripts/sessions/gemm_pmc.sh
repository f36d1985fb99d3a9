set -e
cd "$GRAFT_REPO_ROOT"
for c in "dwo 1282 8" "dwo 1282 16" "dwo_slabs 1282 8" "dwo_slabs 1282 16" "dwqkv 1282 8" "qkv 2561" "qkv 1282"; do
  timeout -k 10 60 python scripts/gemm_one.py $c
done > gpurun_out/one.log 2>&1
scripts/pmc_gemm.sh gpurun_out/pmcg "dwo 1282 8" "dwo_slabs 1282 8" "qkv 2561 1" > gpurun_out/pmc.log 2>&1
