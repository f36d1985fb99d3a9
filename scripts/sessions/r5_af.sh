# grouped weight-gradient pair with the half-slot 1282 pick at T <= 4096: e2e bit-exact tests,
# then B=8 x3 and B=64 x2 interleaved (LJS_DW_GROUP=1 default vs 0) and a B=8 kernel trace
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r5af
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
step $O/tests.txt timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_e2e.py tests/test_kernels_gpu.py -k "gemm_group or e2e or bit_exact or slab or adam"
for rep in 1 2 3; do
  step $O/b8_group_$rep.txt timeout -k 10 300 python bench.py --batch-per-gpu 8
  LJS_DW_GROUP=0 step $O/b8_sep_$rep.txt timeout -k 10 300 python bench.py --batch-per-gpu 8
done
for rep in 1 2; do
  step $O/b64_group_$rep.txt timeout -k 10 300 python bench.py
  LJS_DW_GROUP=0 step $O/b64_sep_$rep.txt timeout -k 10 300 python bench.py
done
cd /tmp && step $O/prof_b8.txt timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_b8 -o run -- python $R/bench.py --batch-per-gpu 8 --steps 20 --warmup 5
echo done
