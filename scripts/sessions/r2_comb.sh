set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_epilogue_gpu.py tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k "combine or slab or linear or gemm" > gpurun_out/r2m_tests.log 2>&1
timeout -k 10 200 python bench.py --steps 200 --warmup 20 --batch-per-gpu 8 > gpurun_out/r2m_b8.log 2>&1
LJS_DW_COMBINE=0 timeout -k 10 200 python bench.py --steps 200 --warmup 20 --batch-per-gpu 8 > gpurun_out/r2m_b8_nocomb.log 2>&1
timeout -k 10 200 python bench.py --steps 200 --warmup 20 --batch-per-gpu 8 > gpurun_out/r2m_b8_2.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r2m_prof -o prof -- python bench.py --steps 100 --warmup 10 --batch-per-gpu 8 > gpurun_out/r2m_prof.log 2>&1
