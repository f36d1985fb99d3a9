# the weight-gradient pair on the 8-wave tiles at one round of 256 slots (3 + 3 splits) vs the
# 1282 pair (6 + 6), T = 16384 and T = 2048, graph-timed
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$PWD/gpurun_out/r5au
mkdir -p $O
T=16384 timeout -k 10 300 python scripts/gemm_cases.py dwgroup_8w > $O/t16384.txt 2>&1 &&
T=2048 timeout -k 10 300 python scripts/gemm_cases.py dwgroup_8w > $O/t2048.txt 2>&1 && echo done
