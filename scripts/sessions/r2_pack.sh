set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py tests/test_gpu_e2e.py -x -q --timeout 200 --timeout-method thread -k "pack or e2e or mesh or virtual" > gpurun_out/r2pk_tests.log 2>&1
timeout -k 10 200 env LJS_NUM_DEVICES=4 python bench.py --steps 20 --warmup 5 --model fsdp --mesh 4x1 > gpurun_out/r2pk_fsdp4.log 2>&1
timeout -k 10 200 env LJS_NUM_DEVICES=4 python bench.py --steps 20 --warmup 5 --mesh 2d > gpurun_out/r2pk_2d.log 2>&1
