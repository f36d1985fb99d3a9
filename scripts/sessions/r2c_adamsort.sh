set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -q -x -k "adam or deferred or bit_exact" --timeout 120 --timeout-method thread > gpurun_out/r2c_adamsort_tests.log 2>&1
LJS_ADAM_SG=8 timeout -k 10 300 python -u -m pytest tests -m gpu -q -x -k "adam or deferred or bit_exact" --timeout 120 --timeout-method thread >> gpurun_out/r2c_adamsort_tests.log 2>&1
out=gpurun_out/r2c_adamsort.log
for rep in 1 2 3; do
for cfg in "LJS_ADAM_SORT=0" "LJS_ADAM_SORT=1" "LJS_ADAM_SG=8"; do
  for a in "" "--batch-per-gpu 8"; do
    r=$(env $cfg timeout -k 10 120 python bench.py --steps 100 --warmup 20 $a | tail -1 | python -c "import json,sys; print(json.loads(sys.stdin.read())['ms_per_step'])")
    echo "$cfg [$a] $r" >> $out
  done
done
done
for cfg in "LJS_ADAM_SORT=0" "LJS_ADAM_SORT=1" "LJS_ADAM_SG=8"; do
  env $cfg timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r2c_as_$cfg -o prof -- python bench.py --steps 20 --warmup 5 > /dev/null 2>&1
done
