set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/r2c_gs.log
for rep in 1 2 3; do
for G in 1 2 4 8; do
  for a in "--batch-per-gpu 8" ""; do
    r=$(timeout -k 10 120 python bench.py --steps 96 --warmup 16 --graph-steps $G $a | tail -1 | python -c "import json,sys; print(json.loads(sys.stdin.read())['ms_per_step'])")
    echo "G=$G [$a] $r" >> $out
  done
done
done
