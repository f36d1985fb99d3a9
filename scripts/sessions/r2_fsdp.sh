set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_dense_paths_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2f_dense.log 2>&1
timeout -k 10 200 python bench.py --model fsdp --steps 30 --warmup 5 > gpurun_out/r2f_fsdp1.log 2>&1
LJS_NUM_DEVICES=4 timeout -k 10 200 python bench.py --model fsdp --steps 30 --warmup 5 > gpurun_out/r2f_fsdp4.log 2>&1
LJS_NUM_DEVICES=4 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/r2f_prof4 -o prof -- python bench.py --model fsdp --steps 10 --warmup 3 > gpurun_out/r2f_prof4.log 2>&1
