set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py tests/test_epilogue_gpu.py -x -q --timeout 200 --timeout-method thread -k "fp8 or ff_block or layer or side_stream or adam or weight_grad" > gpurun_out/r2sd_tests.log 2>&1
o=gpurun_out/r2sd_ab.txt
: > $o
for i in 1 2; do
for f in 0 1; do
  for m in "" "--batch-per-gpu 8" "--model layer" "--model layer --fp8"; do
    echo "side=$f $m $(LJS_SIDE_WGRAD=$f timeout -k 10 200 python bench.py --steps 100 --warmup 20 $m 2>&1 | grep -o '"ms_per_step": [0-9.]*')" >> $o
  done
done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r2sd_prof8 -o prof -- python bench.py --steps 20 --warmup 5 --batch-per-gpu 8 > gpurun_out/r2sd_prof8.log 2>&1
