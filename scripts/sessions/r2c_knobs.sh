set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/r2c_knobs.log
for rep in 1 2; do
for cfg in "X=0" "LJS_DW_TRAFFIC_W=2" "LJS_DW_TRAFFIC_W=4" "LJS_DW_TRAFFIC_W=0.5" "LJS_ADAM_ROWS=32"; do
  for a in "" "--batch-per-gpu 8"; do
    r=$(env $cfg timeout -k 10 120 python bench.py --steps 100 --warmup 20 $a | tail -1 | python -c "import json,sys; print(json.loads(sys.stdin.read())['ms_per_step'])")
    echo "$cfg [$a] $r" >> $out
  done
done
done
