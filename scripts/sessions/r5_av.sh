# the 8-wave weight-gradient pair at T <= 4096 (B=8: 3 + 3 splits on 12884): group tests, B=8 x3
# vs the 1282 6 + 6 pair (LJS_DW_PAIR=6,6,1282), B=64 once, B=8 kernel trace
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r5av
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
step $O/tests.txt timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ -k "gemm_group or grouped or deferred or e2e"
for rep in 1 2 3; do
  step $O/b8_8w_$rep.txt timeout -k 10 300 python bench.py --batch-per-gpu 8
  LJS_DW_PAIR=6,6,1282 step $O/b8_1282_$rep.txt timeout -k 10 300 python bench.py --batch-per-gpu 8
done
step $O/b64.txt timeout -k 10 300 python bench.py
cd /tmp && step $O/prof_b8.txt timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof_b8 -o run -- python $R/bench.py --batch-per-gpu 8 --steps 20 --warmup 5
echo done
