set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 200 python bench.py --steps 50 --warmup 10 > gpurun_out/r2fc_b64.log 2>&1
timeout -k 10 200 python bench.py --steps 200 --warmup 20 --batch-per-gpu 8 > gpurun_out/r2fc_b8.log 2>&1
timeout -k 10 200 python bench.py --steps 50 --warmup 10 --model layer > gpurun_out/r2fc_layer_bf16.log 2>&1
timeout -k 10 200 python bench.py --steps 50 --warmup 10 --model layer --fp8 > gpurun_out/r2fc_layer_fp8.log 2>&1
timeout -k 10 200 python bench.py --steps 50 --warmup 10 --model ff > gpurun_out/r2fc_ff_bf16.log 2>&1
timeout -k 10 200 python bench.py --steps 50 --warmup 10 --model ff --fp8 > gpurun_out/r2fc_ff_fp8.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r2fc_prof -o prof -- python bench.py --steps 20 --warmup 5 --model layer --fp8 > gpurun_out/r2fc_prof.log 2>&1
