set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s3_tiles_tests.log 2>&1
for i in 1 2; do timeout -k 10 200 python bench.py >> gpurun_out/s3_tiles_b64.log 2>&1; done
timeout -k 10 200 python bench.py --model layer --fp8 > gpurun_out/s3_tiles_layer8.log 2>&1
timeout -k 10 200 python bench.py --model layer > gpurun_out/s3_tiles_layer.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof16 -o run -- python bench.py --steps 25 --warmup 5 > gpurun_out/prof16.log 2>&1
