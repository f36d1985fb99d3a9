set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2c_final_tests.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2c_final_smoke.log 2>&1
out=gpurun_out/r2c_final_fused.log
for cfg in "LJS_ATTN_BWD_FUSED=2" "LJS_ATTN_BWD_FUSED=0"; do
  for a in "--batch-per-gpu 16" "--batch-per-gpu 32"; do
    r=$(env $cfg timeout -k 10 120 python bench.py --steps 96 --warmup 16 $a | tail -1 | python -c "import json,sys; print(json.loads(sys.stdin.read())['ms_per_step'])")
    echo "$cfg [$a] $r" >> $out
  done
done
for a in "" "--batch-per-gpu 8" "--seq 4096 --batch-per-gpu 4"; do
  echo "$a $(timeout -k 10 200 python bench.py $a | tail -1)" >> gpurun_out/r2c_final_bench.log
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r2c_final_b8 -o prof -- python bench.py --steps 32 --warmup 8 --batch-per-gpu 8 > /dev/null 2>&1
