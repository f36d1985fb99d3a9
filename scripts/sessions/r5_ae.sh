# grouped weight-gradient GEMM pair (dW_qkv batch + dW_o as one grid) vs separate, by tile and
# split count, at T = 2048 (B = 8) and T = 16384 (B = 64); graph-timed
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$PWD/gpurun_out/r5ae
mkdir -p $O
T=2048 timeout -k 10 240 python scripts/gemm_cases.py dwgroup > $O/dwgroup_t2048.txt 2>&1 &&
T=16384 timeout -k 10 240 python scripts/gemm_cases.py dwgroup > $O/dwgroup_t16384.txt 2>&1 && echo done
