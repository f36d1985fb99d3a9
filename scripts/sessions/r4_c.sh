# ping-pong GEMM v2 (DMA in the MFMA intervals): numerics, A/B timing, then the step with / without it
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r4c
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then case $rc in 1|2) ;; *) exit $rc;; esac; fi; }
step $O/pp_tests.log timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gemm_pp_gpu.py
if grep -q " failed\|Error" $O/pp_tests.log; then echo "pp tests failed"; tail -30 $O/pp_tests.log; exit 1; fi
step $O/pp_bench.log timeout -k 10 300 python scripts/gemm_pp_bench.py
step $O/drv_pp0.log env LJS_GEMM_PP=0 timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5
step $O/drv_pp1.log timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5
step $O/b8.log timeout -k 10 200 python bench.py --batch-per-gpu 8 --steps 20 --warmup 5
cd /tmp
step $O/prof_b64.log timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_b64 -o run -- python3 $R/bench.py --steps 16 --warmup 4
echo done
