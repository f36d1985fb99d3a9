set -e
cd "$GRAFT_REPO_ROOT"
for c in "dwall 1282 8" "dwall 1282 4" "dwall_slabs 1282 8" "dwall_slabs 1282 4" "dwall_kc 1282 8" "dwall_kc 1282 4" "dwall_kc 2561 4" "dwall_kc 2561 8"; do
  timeout -k 10 60 python scripts/gemm_one.py $c
done > gpurun_out/one.log 2>&1
