# the B=8 attention backward variants re-checked on the final build: 128-key dK/dV + 128-query dQ
# blocks (default pair32), 64-query dQ (LJS_ATTN_DQ32=0), 64-key pair kernel (LJS_ATTN_DKV32=0),
# fused per-(b,h) kernel (LJS_ATTN_BWD_FUSED=1); x3 interleaved
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r5bg
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
for rep in 1 2 3; do
  step $O/base_$rep.txt timeout -k 10 300 python bench.py --batch-per-gpu 8
  LJS_ATTN_DQ32=0 step $O/dq64_$rep.txt timeout -k 10 300 python bench.py --batch-per-gpu 8
  LJS_ATTN_DKV32=0 step $O/pair64_$rep.txt timeout -k 10 300 python bench.py --batch-per-gpu 8
  LJS_ATTN_BWD_FUSED=1 step $O/fused_$rep.txt timeout -k 10 300 python bench.py --batch-per-gpu 8
done
echo done
