# driver shape (--steps 20 --warmup 5) by graph length on the final build: G = 5 (default rule),
# 4, 10; B=64 x3 interleaved
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r5bh
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
for rep in 1 2 3; do
  for g in 5 4 10; do
    step $O/b64_g${g}_$rep.txt timeout -k 10 300 python bench.py --steps 20 --warmup 5 --graph-steps $g
  done
done
echo done
