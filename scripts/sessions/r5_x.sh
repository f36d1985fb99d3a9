# reference shape (B=8) levers: weight-gradient tile / split variants at T = 2048 (isolated), and
# the 2-block 1282 weight-gradient tiles at T = 2048 (LJS_DW_SMALL_TILE=1282), and
# Adam's tile-height threshold (LJS_ADAM_SPLIT_S 8: 32-row tiles for W_o's 12 slabs) A/B
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r5x
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
T=2048 step $O/dw_t2048.txt timeout -k 10 300 python scripts/gemm_cases.py dwqkv_ring dwo_ring qkv dh out
for rep in 1 2 3; do
  step $O/b8_default_$rep.txt timeout -k 10 300 python bench.py --batch-per-gpu 8
  LJS_ADAM_SPLIT_S=8 step $O/b8_split8_$rep.txt timeout -k 10 300 python bench.py --batch-per-gpu 8
  LJS_DW_SMALL_TILE=1282 step $O/b8_dw1282_$rep.txt timeout -k 10 300 python bench.py --batch-per-gpu 8
done
echo done
