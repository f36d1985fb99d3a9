# round 5 session start: new GPU tests (real-backend multi-device capture, zero-stride MX proxy),
# the driver-shape line, and the slow-start trace (per-step kernel durations, steps 1..N)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r5a
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then case $rc in 1|2) ;; *) exit $rc;; esac; fi; }
step $O/tests.log timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_multi_gpu_capture_gpu.py "tests/test_gpu_e2e.py::test_jit_graph_train_step_matches_eager" \
  "tests/test_gpu_e2e.py::test_fp8_ff_block_2d_gathers_mx_shadows"
step $O/drv.log timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5
step $O/drv_nomin.log timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --min-warmup 0
step $O/drv_nomin_g1.log timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --min-warmup 0 --graph-steps 1
cd /tmp
step $O/ramp.log timeout -k 10 300 rocprofv3 --kernel-trace -d $O/ramp -o run -- python3 $R/bench.py --steps 80 --warmup 5 --min-warmup 0 --graph-steps 1
cd $R
python scripts/step_ramp.py $(ls $O/ramp/*/run_results.db $O/ramp/run_results.db 2>/dev/null | head -1) --out $O/ramp.md > /dev/null 2>&1 || true
python scripts/kernel_resources.py --grep gemm_dma > $O/gemm_regs.txt 2>&1 || true
echo done
