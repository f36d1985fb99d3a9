# lean K-loop GEMM: bit-exactness and A/B against the general LDS-DMA kernel
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$PWD/gpurun_out/r5f
mkdir -p $O
LJS_GEMM_LEAN=0 timeout -k 10 300 python scripts/gemm_lean_ab.py > $O/lean.log 2>&1
echo rc=$?
