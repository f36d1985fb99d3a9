set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x -k "cast_on_load" --timeout 120 --timeout-method thread > gpurun_out/r2c_col_tests.log 2>&1
out=gpurun_out/r2c_col.log
for rep in 1 2 3; do
for cfg in "LJS_CAST_ON_LOAD=0" "LJS_CAST_ON_LOAD=1"; do
  for a in "--batch-per-gpu 8" "--batch-per-gpu 16" ""; do
    r=$(env $cfg timeout -k 10 120 python bench.py --steps 100 --warmup 20 $a | tail -1 | python -c "import json,sys; print(json.loads(sys.stdin.read())['ms_per_step'])")
    echo "$cfg [$a] $r" >> $out
  done
done
done
LJS_CAST_ON_LOAD=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r2c_col_b8 -o prof -- python bench.py --steps 20 --warmup 5 --batch-per-gpu 8 > /dev/null 2>&1
