set -e
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q -k fp8 > gpurun_out/kern.log 2>&1
timeout -k 10 400 python -m pytest tests/test_gpu_e2e.py -x -q -k fp8 > gpurun_out/e2e.log 2>&1
timeout -k 10 200 python bench.py --model layer --steps 30 --warmup 5 > gpurun_out/bench_layer.log 2>&1
timeout -k 10 200 python bench.py --model layer --fp8 --steps 30 --warmup 5 > gpurun_out/bench_layer_fp8.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_fp8" -- python3 "$GRAFT_REPO_ROOT/bench.py" --model layer --fp8 --steps 20 --warmup 5 > "$GRAFT_REPO_ROOT/gpurun_out/prof_fp8.log" 2>&1
