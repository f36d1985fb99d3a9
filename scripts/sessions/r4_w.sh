# out-projection: compile-time bias + fused-sum epilogue instance (RES 4; LJS_GEMM_BSUM=0 off)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r4w
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then case $rc in 1|2) ;; *) exit $rc;; esac; fi; }
step $O/tests.log timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_epilogue_gpu.py tests/test_dense_paths_gpu.py tests/test_gpu_e2e.py
if grep -q " failed\|[0-9] error" $O/tests.log; then echo "tests failed"; tail -30 $O/tests.log; exit 1; fi
for i in 1 2 3; do
step $O/gemm_b1_$i.log timeout -k 10 200 python scripts/gemm_ab.py out
step $O/gemm_b0_$i.log env LJS_GEMM_BSUM=0 timeout -k 10 200 python scripts/gemm_ab.py out
done
for i in 1 2 3; do
step $O/b64_b1_$i.log timeout -k 10 200 python bench.py --steps 20 --warmup 5
step $O/b64_b0_$i.log env LJS_GEMM_BSUM=0 timeout -k 10 200 python bench.py --steps 20 --warmup 5
step $O/b8_b1_$i.log timeout -k 10 200 python bench.py --batch-per-gpu 8 --steps 20 --warmup 5
step $O/b8_b0_$i.log env LJS_GEMM_BSUM=0 timeout -k 10 200 python bench.py --batch-per-gpu 8 --steps 20 --warmup 5
done
for f in $O/b*.log; do grep -h ms_per_step $f | python -c "
import sys,json
for l in sys.stdin:
    r=json.loads(l); print('$(basename $f)', r['ms_per_step'])
" >> $O/summary.txt || true; done
echo done
