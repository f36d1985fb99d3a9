set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s3_fin_tests.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s3_fin_smoke.log 2>&1
for i in 1 2; do timeout -k 10 200 python bench.py >> gpurun_out/s3_fin_b64.log 2>&1; done
timeout -k 10 200 python bench.py --batch-per-gpu 8 > gpurun_out/s3_fin_b8.log 2>&1
timeout -k 10 200 python bench.py --mode fwd > gpurun_out/s3_fin_fwd.log 2>&1
WORLD_SIZE=8 RANK=0 LOCAL_RANK=0 LJS_DIST_BACKEND=fake MASTER_ADDR=127.0.0.1 MASTER_PORT=29555 timeout -k 10 200 python bench.py --gpus 8 > gpurun_out/s3_fin_w8.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof15 -o run -- python bench.py --steps 25 --warmup 5 > gpurun_out/prof15.log 2>&1
