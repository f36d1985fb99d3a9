set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
o=gpurun_out/r2defer.txt
: > $o
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_epilogue_gpu.py -k "deferred or side_stream" > gpurun_out/r2defer_tests.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r2defer_b64 -o prof -- python bench.py --steps 20 --warmup 5 > gpurun_out/r2defer_b64.log 2>&1
for i in 1 2; do
  echo "b64 $(timeout -k 10 200 python bench.py --steps 200 --warmup 20 2>&1 | grep -o '"ms_per_step": [0-9.]*')" >> $o
  echo "b8 $(timeout -k 10 200 python bench.py --steps 200 --warmup 20 --batch-per-gpu 8 2>&1 | grep -o '"ms_per_step": [0-9.]*')" >> $o
  echo "b64-nodefer $(LJS_DEFER_WGRAD=0 timeout -k 10 200 python bench.py --steps 200 --warmup 20 2>&1 | grep -o '"ms_per_step": [0-9.]*')" >> $o
  echo "b8-nodefer $(LJS_DEFER_WGRAD=0 timeout -k 10 200 python bench.py --steps 200 --warmup 20 --batch-per-gpu 8 2>&1 | grep -o '"ms_per_step": [0-9.]*')" >> $o
done
