# compile-time plain epilogue (RES 3: alpha 1, no bias / ReLU / fused sum; LJS_GEMM_PLAIN=0 for the
# general kernel) for the QKV / dX GEMMs; the 256x192 QKV tile (LJS_GEMM_TILE2562=1); this build vs
# the session-start build (nopin variant); numerics, isolated A/B, steps at B=64 / B=8, tables
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r4s
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then case $rc in 1|2) ;; *) exit $rc;; esac; fi; }
step $O/tests.log timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_epilogue_gpu.py tests/test_dense_paths_gpu.py
if grep -q " failed\|[0-9] error" $O/tests.log; then echo "tests failed"; tail -30 $O/tests.log; exit 1; fi
for i in 1 2 3; do
step $O/gemm_plain_$i.log timeout -k 10 200 python scripts/gemm_ab.py qkv qkv:2562 dh
step $O/gemm_gen_$i.log env LJS_GEMM_PLAIN=0 timeout -k 10 200 python scripts/gemm_ab.py qkv qkv:2562 dh
step $O/gemm_nopin_$i.log env LJS_KERNELS_LIB=$R/learning_jax_sharding_amd/_lib/variants/nopin/libljs_kernels.so timeout -k 10 200 python scripts/gemm_ab.py qkv out dh
done
for i in 1 2 3; do
step $O/b64_plain_$i.log timeout -k 10 200 python bench.py --steps 20 --warmup 5
step $O/b64_gen_$i.log env LJS_GEMM_PLAIN=0 timeout -k 10 200 python bench.py --steps 20 --warmup 5
step $O/b64_t2562_$i.log env LJS_GEMM_TILE2562=1 timeout -k 10 200 python bench.py --steps 20 --warmup 5
step $O/b8_plain_$i.log timeout -k 10 200 python bench.py --batch-per-gpu 8 --steps 20 --warmup 5
step $O/b8_gen_$i.log env LJS_GEMM_PLAIN=0 timeout -k 10 200 python bench.py --batch-per-gpu 8 --steps 20 --warmup 5
step $O/b64_nopin_$i.log env LJS_KERNELS_LIB=$R/learning_jax_sharding_amd/_lib/variants/nopin/libljs_kernels.so timeout -k 10 200 python bench.py --steps 20 --warmup 5
step $O/b8_nopin_$i.log env LJS_KERNELS_LIB=$R/learning_jax_sharding_amd/_lib/variants/nopin/libljs_kernels.so timeout -k 10 200 python bench.py --batch-per-gpu 8 --steps 20 --warmup 5
done
cd /tmp
step $O/prof_b64.log timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_b64 -o run -- python3 $R/bench.py --steps 16 --warmup 4
step $O/prof_b8.log timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_b8 -o run -- python3 $R/bench.py --batch-per-gpu 8 --steps 16 --warmup 4
cd $R
for p in prof_b64 prof_b8; do
  n=$(grep -h ms_per_step $O/$p.log | python -c "import sys,json; r=json.loads(sys.stdin.readline()); print(r['warmup']+r['steps'])")
  python scripts/kstats.py $(ls $O/$p/*/run_results.db $O/$p/run_results.db 2>/dev/null | head -1) --steps $n --title "$p" --out $O/$p.md || true
done
for f in $O/b*.log; do grep -h ms_per_step $f | python -c "
import sys,json
for l in sys.stdin:
    r=json.loads(l); print('$(basename $f)', r['ms_per_step'])
" >> $O/summary.txt || true; done
echo done
