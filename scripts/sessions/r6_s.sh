# round-6: phase timing of the fused attention backward (diagnostic build)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r6s
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
step $O/bwd_phases.txt timeout -k 10 120 env LJS_KERNELS_LIB=$R/learning_jax_sharding_amd/_lib/variants/bwdtrace/libljs_kernels.so python scripts/attn_bwd_phases.py 64
step $O/fwd_phases.txt timeout -k 10 120 env LJS_KERNELS_LIB=$R/learning_jax_sharding_amd/_lib/variants/qatrace/libljs_kernels.so python scripts/qkv_attn_phases.py 64
echo done
