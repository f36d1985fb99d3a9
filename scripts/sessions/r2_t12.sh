set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_epilogue_gpu.py tests/test_dense_paths_gpu.py -x -q --timeout 200 --timeout-method thread -k "cast_on_load or gemm or linear or dense or transformer" > gpurun_out/r2t12_tests.log 2>&1
o=gpurun_out/r2t12.txt
: > $o
for i in 1 2 3; do
  for m in "" "--batch-per-gpu 8"; do
    echo "$m $(timeout -k 10 200 python bench.py --steps 100 --warmup 20 $m 2>&1 | grep -o '"ms_per_step": [0-9.]*')" >> $o
  done
done
