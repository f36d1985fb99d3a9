set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s3_full3_tests.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s3_full3_smoke.log 2>&1
timeout -k 10 200 python bench.py > gpurun_out/s3_full3_bench.log 2>&1
for w in 2 8; do
WORLD_SIZE=$w RANK=0 LOCAL_RANK=0 LJS_DIST_BACKEND=fake MASTER_ADDR=127.0.0.1 MASTER_PORT=29555 timeout -k 10 200 python bench.py --steps 50 --warmup 10 --gpus $w > gpurun_out/s3_reh_w$w.log 2>&1
done
