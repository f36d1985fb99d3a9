# driver shape (--steps 20 --warmup 5) by graph length: G = 4 / 5 (default) / 10 / 20, x3
# interleaved, B=64 and B=8
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r5ap
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
for rep in 1 2 3; do
  for g in 4 5 10 20; do
    step $O/b64_g${g}_$rep.txt timeout -k 10 300 python bench.py --steps 20 --warmup 5 --graph-steps $g
    step $O/b8_g${g}_$rep.txt timeout -k 10 300 python bench.py --steps 20 --warmup 5 --graph-steps $g --batch-per-gpu 8
  done
done
echo done
