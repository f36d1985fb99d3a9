set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_epilogue_gpu.py -x -q --timeout 200 --timeout-method thread -k "gemm or linear or epilogue" > gpurun_out/r2b8_tests.log 2>&1
timeout -k 10 200 python bench.py --steps 200 --warmup 20 --batch-per-gpu 8 > gpurun_out/r2b8_def.log 2>&1
LJS_ATTN_FWD_RES=4 timeout -k 10 200 python bench.py --steps 200 --warmup 20 --batch-per-gpu 8 > gpurun_out/r2b8_res4.log 2>&1
LJS_ATTN_FWD_RES=0 timeout -k 10 200 python bench.py --steps 200 --warmup 20 --batch-per-gpu 8 > gpurun_out/r2b8_res0.log 2>&1
timeout -k 10 200 python bench.py --steps 50 --warmup 10 > gpurun_out/r2b8_b64.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r2b8_prof -o prof -- python bench.py --steps 100 --warmup 10 --batch-per-gpu 8 > gpurun_out/r2b8_prof.log 2>&1
