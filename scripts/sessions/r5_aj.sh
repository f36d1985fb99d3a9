# Adam tile height after the pair split change (6 + 6 slabs for every weight): 64 (default) vs
# 32 vs 16-row tiles, B=64 and B=8 x3 interleaved
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r5aj
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
for rep in 1 2 3; do
  for rows in 64 32 16; do
    LJS_ADAM_ROWS=$rows step $O/b64_r${rows}_$rep.txt timeout -k 10 300 python bench.py
    LJS_ADAM_ROWS=$rows step $O/b8_r${rows}_$rep.txt timeout -k 10 300 python bench.py --batch-per-gpu 8
  done
done
echo done
