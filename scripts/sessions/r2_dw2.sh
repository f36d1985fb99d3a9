set -e
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r2dw2.log
: > $o
for cfg in "dwslab:640:1536 1282 8" "dwslab:640:1536 2563 7" "dwslab:640:1536 12856 8" "dwslab:640:1536 12856 16" \
           "dwslab:2560:640 1282 5" "dwslab:2560:640 2563 5" "dwslab:2560:640 2563 10" "dwslab:2560:640 12856 4" \
           "dwslab:640:2560 1282 5" "dwslab:640:2560 2563 4" "dwslab:640:2560 12856 5" "dwslab:640:2560 12856 10" \
           "dwslab:512:640 1282 24" "dwslab:512:640 2563 24" "dwslab:512:640 12856 20"; do
  timeout -k 10 120 python scripts/gemm_one.py $cfg 50 2>&1 | grep -v amdgpu.ids >> $o
done
