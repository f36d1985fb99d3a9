set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_gpu_e2e.py -q -x -k "attention or e2e or ring or sequence" --timeout 120 --timeout-method thread > gpurun_out/s3_pk_tests.log 2>&1
timeout -k 10 100 python scripts/attn_bench.py > gpurun_out/s3_pk_attn.log 2>&1
timeout -k 10 200 python bench.py > gpurun_out/s3_pk_b64.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof14 -o run -- python bench.py --steps 25 --warmup 5 > gpurun_out/prof14.log 2>&1
