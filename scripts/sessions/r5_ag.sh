# fewer weight-gradient slabs at T = 2048 (B = 8): 64x64 tiles at 1 / 2 splits (320 / 640 items
# over the pair) vs the grouped 1282 pair (4 + 11 splits); isolated, graph-timed
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$PWD/gpurun_out/r5ag
mkdir -p $O
T=2048 timeout -k 10 240 python scripts/gemm_cases.py dwgroup dwqkv_ring dwo_ring > $O/t2048.txt 2>&1 && echo done
