# grouped weight-gradient pair at T = 16384 (B = 64) with fewer, longer splits (one round of
# resident blocks for the pair instead of two full-chip launches): GEMM time by split pair
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$PWD/gpurun_out/r5ah
mkdir -p $O
T=16384 timeout -k 10 300 python scripts/gemm_cases.py dwgroup_big > $O/t16384.txt 2>&1 && echo done
