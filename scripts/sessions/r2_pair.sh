set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
o=gpurun_out/r2pair.txt
: > $o
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "attention or attn" > gpurun_out/r2pair_tests.log 2>&1
for i in 1 2; do
  echo "pair $(timeout -k 10 120 python scripts/attn_time.py 8 256 8 2>&1 | tail -1)" >> $o
  echo "nopair $(LJS_ATTN_BWD_PAIR=0 timeout -k 10 120 python scripts/attn_time.py 8 256 8 2>&1 | tail -1)" >> $o
  echo "b8 pair $(timeout -k 10 200 python bench.py --steps 200 --warmup 20 --batch-per-gpu 8 2>&1 | grep -o '"ms_per_step": [0-9.]*')" >> $o
  echo "b8 nopair $(LJS_ATTN_BWD_PAIR=0 timeout -k 10 200 python bench.py --steps 200 --warmup 20 --batch-per-gpu 8 2>&1 | grep -o '"ms_per_step": [0-9.]*')" >> $o
  echo "b16 pair $(timeout -k 10 200 python bench.py --steps 200 --warmup 20 --batch-per-gpu 16 2>&1 | grep -o '"ms_per_step": [0-9.]*')" >> $o
  echo "b16 nopair $(LJS_ATTN_BWD_PAIR=0 timeout -k 10 200 python bench.py --steps 200 --warmup 20 --batch-per-gpu 16 2>&1 | grep -o '"ms_per_step": [0-9.]*')" >> $o
done
