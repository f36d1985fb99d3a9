set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2c_last_tests.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2c_last_smoke.log 2>&1
for a in "" "--batch-per-gpu 8" "--seq 4096 --batch-per-gpu 4" "--model layer --fp8"; do
  echo "$a $(timeout -k 10 200 python bench.py $a | tail -1)" >> gpurun_out/r2c_last_bench.log
done
