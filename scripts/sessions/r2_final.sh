set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2fin_tests.log 2>&1
o=gpurun_out/r2fin_bench.txt
: > $o
for m in "" "--batch-per-gpu 8" "--model layer" "--model layer --fp8" "--model ff" "--model ff --fp8" "--model fsdp"; do
  echo "$m $(timeout -k 10 200 python bench.py --steps 100 --warmup 20 $m 2>&1 | tail -1)" >> $o
done
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2fin_smoke.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r2fin_b64 -o prof -- python bench.py --steps 20 --warmup 5 > gpurun_out/r2fin_b64.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r2fin_b8 -o prof -- python bench.py --steps 20 --warmup 5 --batch-per-gpu 8 > gpurun_out/r2fin_b8.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r2fin_layer -o prof -- python bench.py --steps 20 --warmup 5 --model layer > gpurun_out/r2fin_layer.log 2>&1
