# round-6: the fused attention phase software-pipelined by two key tiles (score MFMAs of tile kt+1 before the softmax of kt)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r6n
mkdir -p $O
V=$R/learning_jax_sharding_amd/_lib/variants
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
step $O/tests_k.txt timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "qkv_attn"
step $O/tests_e.txt timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_e2e.py -k "fused_qkv"
step $O/phases_pipe.txt timeout -k 10 120 env LJS_KERNELS_LIB=$V/qatrace/libljs_kernels.so python scripts/qkv_attn_phases.py 64
step $O/phases_nopipe.txt timeout -k 10 120 env LJS_KERNELS_LIB=$V/qatrace_nopipe/libljs_kernels.so python scripts/qkv_attn_phases.py 64
for rep in 1 2 3; do
  step $O/b64_pipe_$rep.txt timeout -k 10 300 python bench.py --steps 20 --warmup 5
  step $O/b64_nopipe_$rep.txt timeout -k 10 300 env LJS_KERNELS_LIB=$V/nopipe/libljs_kernels.so python bench.py --steps 20 --warmup 5
done
for f in $O/b*_*.txt; do echo "$(basename $f) $(grep -o '"ms_per_step": [0-9.]*' $f)"; done > $O/lines.txt
echo done
