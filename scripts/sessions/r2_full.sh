set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2full_tests.log 2>&1
o=gpurun_out/r2full_bench.txt
: > $o
for m in "" "--batch-per-gpu 8" "--model layer" "--model layer --fp8" "--model ff" "--model ff --fp8" "--model fsdp"; do
  echo "$m $(timeout -k 10 200 python bench.py --steps 100 --warmup 20 $m 2>&1 | grep -o '"ms_per_step": [0-9.]*')" >> $o
done
echo "fsdp4 $(timeout -k 10 200 env LJS_NUM_DEVICES=4 python bench.py --steps 20 --warmup 5 --model fsdp --mesh 4x1 2>&1 | grep -o '"ms_per_step": [0-9.]*')" >> $o
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2full_smoke.log 2>&1
