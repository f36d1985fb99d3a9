set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_epilogue_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r2e_tests.log 2>&1
timeout -k 10 200 python bench.py --steps 50 --warmup 10 --model layer > gpurun_out/r2e_layer.log 2>&1
timeout -k 10 200 python bench.py --steps 50 --warmup 10 --model ff > gpurun_out/r2e_ff.log 2>&1
timeout -k 10 200 python bench.py --steps 50 --warmup 10 > gpurun_out/r2e_bench64.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r2e_proflayer -o prof -- python bench.py --steps 20 --warmup 5 --model layer > gpurun_out/r2e_proflayer.log 2>&1
