# the 128x96 lean tile for the 2048-token Q/K/V projection: bit-exact test, isolated timing
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$PWD/gpurun_out/r5az
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "128x96 or lean_bit_exact" > $O/tests.txt 2>&1 &&
T=2048 timeout -k 10 240 python scripts/gemm_cases.py qkv_small > $O/qkv_small.txt 2>&1 && echo done
