set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof11 -o run -- python bench.py --steps 25 --warmup 5 > gpurun_out/prof11.log 2>&1
timeout -k 10 200 python bench.py --batch-per-gpu 8 > gpurun_out/s3_b8.log 2>&1
timeout -k 10 200 python bench.py --mode fwd > gpurun_out/s3_fwd.log 2>&1
timeout -k 10 200 python bench.py --model layer > gpurun_out/s3_layer.log 2>&1
timeout -k 10 200 python bench.py --model layer --fp8 > gpurun_out/s3_layer_fp8.log 2>&1
