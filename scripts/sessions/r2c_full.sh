set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2c_gputests.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2c_smoke.log 2>&1
for a in "" "--batch-per-gpu 8" "--model layer" "--model layer --fp8"; do
  echo "$a $(timeout -k 10 200 python bench.py $a | tail -1)" >> gpurun_out/r2c_bench.log
done
