set -e
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "gemm" > gpurun_out/slab_tests.log 2>&1
timeout -k 10 300 python scripts/gemm_study.py > gpurun_out/gemm_study_slab.log 2>&1
timeout -k 10 200 python bench.py --steps 50 --warmup 10 > gpurun_out/bench_slab.log 2>&1
