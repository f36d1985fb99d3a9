set -e
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k "adam or attention" > gpurun_out/r2a_tests.log 2>&1
LJS_ADAM_ROWS=16 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k "adam" > gpurun_out/r2a_tests16.log 2>&1
for r in 64 32 16; do
LJS_ADAM_ROWS=$r timeout -k 10 200 python bench.py --steps 200 --warmup 20 --batch-per-gpu 8 > gpurun_out/r2a_b8_$r.log 2>&1
LJS_ADAM_ROWS=$r timeout -k 10 200 python bench.py --steps 50 --warmup 10 > gpurun_out/r2a_b64_$r.log 2>&1
done
