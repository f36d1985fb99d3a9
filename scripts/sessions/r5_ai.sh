# weight-gradient pair with jointly chosen split counts (hip.pick_dw_pair: one round, 6 + 6 splits
# at both shapes): tests, then B=64 x3 (pair vs LJS_DW_GROUP=0) and B=8 x3 (pair 6/6 vs 11/4 vs
# off) interleaved, and B=64 / B=8 kernel traces
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r5ai
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
step $O/tests.txt timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_e2e.py tests/test_kernels_gpu.py tests/test_dense_paths_gpu.py -k "gemm_group or e2e or bit_exact or slab or adam or dense or attention_block"
for rep in 1 2 3; do
  step $O/b64_pair_$rep.txt timeout -k 10 300 python bench.py
  LJS_DW_GROUP=0 step $O/b64_sep_$rep.txt timeout -k 10 300 python bench.py
  step $O/b8_pair66_$rep.txt timeout -k 10 300 python bench.py --batch-per-gpu 8
  LJS_DW_PAIR=11,4 step $O/b8_pair114_$rep.txt timeout -k 10 300 python bench.py --batch-per-gpu 8
  LJS_DW_GROUP=0 step $O/b8_sep_$rep.txt timeout -k 10 300 python bench.py --batch-per-gpu 8
done
cd /tmp && step $O/prof_b64.txt timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_b64 -o run -- python $R/bench.py --steps 20 --warmup 5
step $O/prof_b8.txt timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_b8 -o run -- python $R/bench.py --batch-per-gpu 8 --steps 20 --warmup 5
echo done
