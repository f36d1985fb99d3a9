# round-6: phase timing of the fused Q/K/V + attention kernel (diagnostic build)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r6l
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
step $O/tests_k.txt timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "qkv_attn"
step $O/phases.txt timeout -k 10 120 env LJS_KERNELS_LIB=$R/learning_jax_sharding_amd/_lib/variants/qatrace/libljs_kernels.so python scripts/qkv_attn_phases.py 64
echo done
