set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
LJS_DW_BIG_TILE=644 timeout -k 10 300 python -u -m pytest tests -m gpu -q -x -k "deferred or bit_exact or wgrad or slab" --timeout 120 --timeout-method thread > gpurun_out/r2c_dwbig_tests.log 2>&1
LJS_DW_BIG_TILE=12884 timeout -k 10 300 python -u -m pytest tests -m gpu -q -x -k "deferred or bit_exact or wgrad or slab" --timeout 120 --timeout-method thread >> gpurun_out/r2c_dwbig_tests.log 2>&1
out=gpurun_out/r2c_dwbig.log
for rep in 1 2 3; do
for cfg in "LJS_DW_BIG_TILE=1282" "LJS_DW_BIG_TILE=644" "LJS_DW_BIG_TILE=12884"; do
  for a in "" "--model layer"; do
    r=$(env $cfg timeout -k 10 120 python bench.py --steps 96 --warmup 16 $a | tail -1 | python -c "import json,sys; print(json.loads(sys.stdin.read())['ms_per_step'])")
    echo "$cfg [$a] $r" >> $out
  done
done
done
for cfg in "LJS_DW_BIG_TILE=644" "LJS_DW_BIG_TILE=12884"; do
  env $cfg timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r2c_dw_$cfg -o prof -- python bench.py --steps 16 --warmup 8 > /dev/null 2>&1
done
