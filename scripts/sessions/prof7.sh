set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_gpu_e2e.py -q -x -k "attention or e2e or ring or sequence" --timeout 120 --timeout-method thread > gpurun_out/attn_tests.log 2>&1
timeout -k 10 200 python bench.py > gpurun_out/bench_xcdattn.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof7 -o run -- python bench.py --steps 25 --warmup 5 > gpurun_out/prof7.log 2>&1
