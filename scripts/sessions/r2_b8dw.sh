set -e
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r2b8dw2.txt
: > $o
export T=2048
for cfg in "dwslab:640:1536 1282 4" "dwslab:640:1536 1282 3" "dwslab:640:1536 1282 5" "dwslab:640:1536 644 1" "dwslab:640:1536 644 2" "dwslab:640:1536 644 3" "dwslab:640:1536 643 2" "dwslab:640:1536 12883 4" "dwslab:640:1536 12884 4" \
           "dwslab:512:640 644 4" "dwslab:512:640 644 6" "dwslab:512:640 644 8" "dwslab:512:640 1282 8" "dwslab:512:640 1282 11" "dwslab:512:640 643 6" "dwslab:512:640 12884 8"; do
  timeout -k 10 60 python scripts/gemm_one.py $cfg 200 2>&1 | grep -v amdgpu.ids >> $o
done
