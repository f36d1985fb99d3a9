cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r6h
mkdir -p $O
timeout -k 10 120 python scripts/qkv_attn_debug.py > $O/debug.txt 2>&1; echo "rc=$?" >> $O/debug.txt
