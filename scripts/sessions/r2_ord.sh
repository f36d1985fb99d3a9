set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
o=gpurun_out/r2o_ab.txt
: > $o
for i in 1 2; do
for ord in "dx,wo,wi" "wi,wo,dx" "wi,dx,wo" "dx,wi,wo"; do
  for f in "" "--fp8"; do
    echo "$ord $f $(LJS_FF_BWD_ORDER=$ord timeout -k 10 200 python bench.py --steps 100 --warmup 20 --model layer $f 2>&1 | grep -o '"ms_per_step": [0-9.]*')" >> $o
  done
done
done
