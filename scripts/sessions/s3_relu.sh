set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_gpu_e2e.py -q -x -k "relu or linear or fp8 or colsum or ticket or layer or e2e" --timeout 120 --timeout-method thread > gpurun_out/s3_relu_tests.log 2>&1
timeout -k 10 200 python bench.py --model layer > gpurun_out/s3_relu_layer.log 2>&1
timeout -k 10 200 python bench.py --model layer --fp8 > gpurun_out/s3_relu_layer8.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_layer2 -o run -- python bench.py --model layer --fp8 --steps 25 --warmup 5 > gpurun_out/prof_layer2.log 2>&1
