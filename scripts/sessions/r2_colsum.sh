set -e
cd "$GRAFT_REPO_ROOT"
LJS_COLSUM=0 timeout -k 10 120 python scripts/colsum_bench.py > gpurun_out/r2c_colsum0.log 2>&1

timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k "colsum or linear or relu or fp8 or sum" > gpurun_out/r2c_tests.log 2>&1
timeout -k 10 200 python bench.py --steps 50 --warmup 10 --model layer > gpurun_out/r2c_layer.log 2>&1
