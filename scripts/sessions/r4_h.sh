# register-staged f32 A (cast-on-load in the 256x128 kernel): numerics, A/B timing, the step with / without
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r4h
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then case $rc in 1|2) ;; *) exit $rc;; esac; fi; }
step $O/tests.log timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "f32_a or cast_on_load or box_slice"
if grep -q " failed\|Error" $O/tests.log; then echo "tests failed"; tail -30 $O/tests.log; exit 1; fi
step $O/qkv32.log timeout -k 10 200 python scripts/gemm_pp_bench.py qkv32 qkv
for i in 1 2; do
step $O/drv_col0_$i.log env LJS_CAST_ON_LOAD=0 timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5
step $O/drv_auto_$i.log timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5
done
step $O/b8_col0.log env LJS_CAST_ON_LOAD=0 timeout -k 10 200 python bench.py --batch-per-gpu 8 --steps 20 --warmup 5
step $O/b8_auto.log timeout -k 10 200 python bench.py --batch-per-gpu 8 --steps 20 --warmup 5
cd /tmp
step $O/prof_b64.log timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_b64 -o run -- python3 $R/bench.py --steps 16 --warmup 4
echo done
