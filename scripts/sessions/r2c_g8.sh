set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_rehearsal_gpu.py tests/test_distributed_gpu.py tests/test_gpu_e2e.py -q -x --timeout 200 --timeout-method thread > gpurun_out/r2c_g8_tests.log 2>&1
for a in "" "--batch-per-gpu 8" "--model layer" "--model layer --fp8" "--model ff" "--model ff --fp8" "--model fsdp"; do
  echo "$a $(timeout -k 10 200 python bench.py $a | tail -1)" >> gpurun_out/r2c_g8_bench.log
done
timeout -k 10 200 python bench.py --steps 7 --warmup 3 | tail -1 >> gpurun_out/r2c_g8_bench.log
