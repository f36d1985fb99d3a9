# 256x192 tile (code 2562, opt-in LJS_GEMM_TILE2562=1) for the QKV projection; plain (alpha 1, no
# bias / ReLU) store loop in the bf16 epilogue (LJS_GEMM_PLAIN_EPI); permlane swap at B=8; numerics, A/B, steps
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r4q
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then case $rc in 1|2) ;; *) exit $rc;; esac; fi; }
V=$R/learning_jax_sharding_amd/_lib/variants
step $O/tests.log timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemm or slab"
if grep -q " failed\|[0-9] error" $O/tests.log; then echo "tests failed"; tail -30 $O/tests.log; exit 1; fi
for i in 1 2 3; do
step $O/gemm_def_$i.log timeout -k 10 200 python scripts/gemm_ab.py qkv qkv:2562 dh
step $O/gemm_noplain_$i.log env LJS_KERNELS_LIB=$V/noplain/libljs_kernels.so timeout -k 10 200 python scripts/gemm_ab.py qkv dh
done
for i in 1 2; do
step $O/b64_def_$i.log timeout -k 10 200 python bench.py --steps 20 --warmup 5
step $O/b64_t2562_$i.log env LJS_GEMM_TILE2562=1 timeout -k 10 200 python bench.py --steps 20 --warmup 5
step $O/b64_noplain_$i.log env LJS_KERNELS_LIB=$V/noplain/libljs_kernels.so timeout -k 10 200 python bench.py --steps 20 --warmup 5
done
for i in 1 2; do
step $O/b8_def_$i.log timeout -k 10 200 python bench.py --batch-per-gpu 8 --steps 20 --warmup 5
step $O/b8_noswap_$i.log env LJS_KERNELS_LIB=$V/noswap/libljs_kernels.so timeout -k 10 200 python bench.py --batch-per-gpu 8 --steps 20 --warmup 5
done
cd /tmp
step $O/prof_b8.log timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_b8 -o run -- python3 $R/bench.py --batch-per-gpu 8 --steps 16 --warmup 4
step $O/prof_b8_noswap.log env LJS_KERNELS_LIB=$V/noswap/libljs_kernels.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_b8_noswap -o run -- python3 $R/bench.py --batch-per-gpu 8 --steps 16 --warmup 4
step $O/prof_b64_t2562.log env LJS_GEMM_TILE2562=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_b64_t2562 -o run -- python3 $R/bench.py --steps 16 --warmup 4
cd $R
for p in prof_b64_t2562 prof_b8 prof_b8_noswap; do
  n=$(grep -h ms_per_step $O/$p.log | python -c "import sys,json; r=json.loads(sys.stdin.readline()); print(r['warmup']+r['steps'])")
  python scripts/kstats.py $(ls $O/$p/*/run_results.db $O/$p/run_results.db 2>/dev/null | head -1) --steps $n --title "$p" --out $O/$p.md || true
done
for f in $O/b*.log; do grep -h ms_per_step $f | python -c "
import sys,json
for l in sys.stdin:
    r=json.loads(l); print('$(basename $f)', r['ms_per_step'])
" >> $O/summary.txt || true; done
echo done
