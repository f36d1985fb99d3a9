# round-6: wider weight-gradient tiles (128x256, 256x128, 256x256) at the step's dW shapes
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r6p
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
step $O/tests.txt timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "weight_grad_slab_tiles"
step $O/wide.txt timeout -k 10 600 python scripts/gemm_cases.py dwqkv_wide dwo_wide
echo done
