set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r2c_b64 -o prof -- python bench.py --steps 20 --warmup 5 > gpurun_out/r2c_b64.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r2c_b8 -o prof -- python bench.py --steps 20 --warmup 5 --batch-per-gpu 8 > gpurun_out/r2c_b8.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r2c_layer -o prof -- python bench.py --steps 20 --warmup 5 --model layer > gpurun_out/r2c_layer.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r2c_layer8 -o prof -- python bench.py --steps 20 --warmup 5 --model layer --fp8 > gpurun_out/r2c_layer8.log 2>&1
