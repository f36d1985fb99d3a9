set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_epilogue_gpu.py -x -q --timeout 200 --timeout-method thread -k "cast_on_load or gemm_layouts or linear or side_stream" > gpurun_out/r2col_tests.log 2>&1
o=gpurun_out/r2col.txt
: > $o
for i in 1 2; do
for f in 0 1; do
  for m in "" "--batch-per-gpu 8"; do
    echo "col=$f $m $(LJS_CAST_ON_LOAD=$f timeout -k 10 200 python bench.py --steps 100 --warmup 20 $m 2>&1 | grep -o '"ms_per_step": [0-9.]*')" >> $o
  done
done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r2col_prof -o prof -- python bench.py --steps 20 --warmup 5 > gpurun_out/r2col_prof.log 2>&1
