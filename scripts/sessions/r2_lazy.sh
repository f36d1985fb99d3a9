set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 200 python bench.py --steps 50 --warmup 10 > gpurun_out/r2l_bench64.log 2>&1
timeout -k 10 200 python bench.py --steps 200 --warmup 20 --batch-per-gpu 8 > gpurun_out/r2l_bench8.log 2>&1
timeout -k 10 200 python bench.py --steps 50 --warmup 10 --model layer > gpurun_out/r2l_layer.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r2l_proflayer -o prof -- python bench.py --steps 20 --warmup 5 --model layer > gpurun_out/r2l_proflayer.log 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2l_gputests.log 2>&1
