set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/r2c_fwdn2.log
for rep in 1 2; do
for cfg in "LJS_ATTN_FWD_NSUB=1" "LJS_ATTN_FWD_NSUB=2"; do
  for a in "--seq 4096 --batch-per-gpu 4" "--seq 1024 --batch-per-gpu 16"; do
    r=$(env $cfg timeout -k 10 120 python bench.py --steps 24 --warmup 8 $a | tail -1 | python -c "import json,sys; print(json.loads(sys.stdin.read())['ms_per_step'])")
    echo "$cfg [$a] $r" >> $out
  done
done
for cfg in "LJS_ATTN_DKV32=-1" "LJS_ATTN_DKV32=1"; do
  for a in "--batch-per-gpu 8" "--batch-per-gpu 16"; do
    r=$(env $cfg timeout -k 10 120 python bench.py --steps 96 --warmup 16 $a | tail -1 | python -c "import json,sys; print(json.loads(sys.stdin.read())['ms_per_step'])")
    echo "$cfg [$a] $r" >> $out
  done
done
done
