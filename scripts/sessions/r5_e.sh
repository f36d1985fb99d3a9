# weight-gradient GEMMs as one round (two streams, fewer slabs) vs the current sequential launches
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$PWD/gpurun_out/r5e
mkdir -p $O
timeout -k 10 200 python scripts/dw_group.py > $O/dw64.log 2>&1 && \
T=2048 timeout -k 10 200 python scripts/dw_group.py > $O/dw8.log 2>&1
echo rc=$?
