# GEMM epilogue: v_permlane16_swap pair exchange (LJS_EPI_PLSWAP) + vector bias loads; numerics,
# isolated A/B (default / base = no permlane swap / nopin = the previous round-4 build), steps
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r4o
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then case $rc in 1|2) ;; *) exit $rc;; esac; fi; }
V=$R/learning_jax_sharding_amd/_lib/variants
step $O/tests.log timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_epilogue_gpu.py tests/test_dense_paths_gpu.py
if grep -q " failed\|[0-9] error" $O/tests.log; then echo "tests failed"; tail -30 $O/tests.log; exit 1; fi
for i in 1 2; do
step $O/gemm_def_$i.log timeout -k 10 200 python scripts/gemm_ab.py
step $O/gemm_base_$i.log env LJS_KERNELS_LIB=$V/base/libljs_kernels.so timeout -k 10 200 python scripts/gemm_ab.py
step $O/gemm_nopin_$i.log env LJS_KERNELS_LIB=$V/nopin/libljs_kernels.so timeout -k 10 200 python scripts/gemm_ab.py
done
for i in 1 2; do
step $O/b64_def_$i.log timeout -k 10 200 python bench.py --steps 20 --warmup 5
step $O/b64_base_$i.log env LJS_KERNELS_LIB=$V/base/libljs_kernels.so timeout -k 10 200 python bench.py --steps 20 --warmup 5
step $O/b64_nopin_$i.log env LJS_KERNELS_LIB=$V/nopin/libljs_kernels.so timeout -k 10 200 python bench.py --steps 20 --warmup 5
step $O/b8_def_$i.log timeout -k 10 200 python bench.py --batch-per-gpu 8 --steps 20 --warmup 5
step $O/b8_nopin_$i.log env LJS_KERNELS_LIB=$V/nopin/libljs_kernels.so timeout -k 10 200 python bench.py --batch-per-gpu 8 --steps 20 --warmup 5
done
step $O/l8_def.log timeout -k 10 200 python bench.py --model layer --fp8 --steps 20 --warmup 5
step $O/l8_nopin.log env LJS_KERNELS_LIB=$V/nopin/libljs_kernels.so timeout -k 10 200 python bench.py --model layer --fp8 --steps 20 --warmup 5
for f in $O/b*.log $O/l*.log; do grep -h ms_per_step $f | python -c "
import sys,json
for l in sys.stdin:
    r=json.loads(l); print('$(basename $f)', r['ms_per_step'])
" >> $O/summary.txt || true; done
echo done
