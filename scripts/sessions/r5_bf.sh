# attention switches re-checked on the final build: static wave priority (LJS_ATTN_PRIO=1) and the
# fused backward's K/V by LDS-DMA at 256 queries (LJS_ATTN_BWD_KV_DMA=1), B=64 x3 interleaved
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r5bf
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
for rep in 1 2 3; do
  step $O/base_$rep.txt timeout -k 10 300 python bench.py
  LJS_ATTN_PRIO=1 step $O/prio_$rep.txt timeout -k 10 300 python bench.py
  LJS_ATTN_BWD_KV_DMA=1 step $O/kvdma_$rep.txt timeout -k 10 300 python bench.py
done
echo done
