# round-6: fused attention backward phases with K / V by register copy (default at 256 queries)
# vs by LDS-DMA beside the first query block; the fused forward's phases
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r6t
mkdir -p $O
V=$R/learning_jax_sharding_amd/_lib/variants
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
step $O/bwd_reg.txt timeout -k 10 120 env LJS_KERNELS_LIB=$V/bwdtrace/libljs_kernels.so python scripts/attn_bwd_phases.py 64
step $O/bwd_dma.txt timeout -k 10 120 env LJS_KERNELS_LIB=$V/bwdtrace/libljs_kernels.so python scripts/attn_bwd_phases.py 64 kvdma
step $O/fwd_phases.txt timeout -k 10 120 env LJS_KERNELS_LIB=$V/qatrace/libljs_kernels.so python scripts/qkv_attn_phases.py 64
echo done
