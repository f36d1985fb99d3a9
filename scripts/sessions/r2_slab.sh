set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k "gemm or slab or weight_grad or linear" > gpurun_out/r2s_tests.log 2>&1
timeout -k 10 200 python bench.py --steps 50 --warmup 10 --model layer > gpurun_out/r2s_layer_bf16.log 2>&1
timeout -k 10 200 python bench.py --steps 50 --warmup 10 > gpurun_out/r2s_b64.log 2>&1
timeout -k 10 200 python bench.py --steps 50 --warmup 10 --batch-per-gpu 8 > gpurun_out/r2s_b8.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r2s_prof -o prof -- python bench.py --steps 20 --warmup 5 --model layer > gpurun_out/r2s_prof.log 2>&1
