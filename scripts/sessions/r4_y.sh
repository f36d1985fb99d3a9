# Adam: the 1-3 remainder slabs' loads ride along with the last 4-slab group (LJS_ADAM_REM_BATCH);
# slab_reduce: every slab's load in one round trip (LJS_SLAB_BATCH); A/B vs the "old" variant
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r4y
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then case $rc in 1|2) ;; *) exit $rc;; esac; fi; }
OLD=$R/learning_jax_sharding_amd/_lib/variants/old/libljs_kernels.so
step $O/tests.log timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_gpu_e2e.py -k "adam or slab or train or optim"
if grep -q " failed\|[0-9] error" $O/tests.log; then echo "tests failed"; tail -30 $O/tests.log; exit 1; fi
F4="WORLD_SIZE=4 RANK=0 LOCAL_RANK=0 LJS_DIST_BACKEND=fake MASTER_ADDR=127.0.0.1"
for i in 1 2 3; do
step $O/b64_new_$i.log timeout -k 10 200 python bench.py --steps 20 --warmup 5
step $O/b64_old_$i.log env LJS_KERNELS_LIB=$OLD timeout -k 10 200 python bench.py --steps 20 --warmup 5
step $O/b8_new_$i.log timeout -k 10 200 python bench.py --batch-per-gpu 8 --steps 20 --warmup 5
step $O/b8_old_$i.log env LJS_KERNELS_LIB=$OLD timeout -k 10 200 python bench.py --batch-per-gpu 8 --steps 20 --warmup 5
done
for i in 1 2; do
step $O/f4dp_new_$i.log env $F4 MASTER_PORT=2983$i timeout -k 10 300 python bench.py --gpus 4 --mesh dp --steps 20 --warmup 5
step $O/f4dp_old_$i.log env $F4 MASTER_PORT=2984$i LJS_KERNELS_LIB=$OLD timeout -k 10 300 python bench.py --gpus 4 --mesh dp --steps 20 --warmup 5
done
cd /tmp
step $O/prof_b64.log timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_b64 -o run -- python3 $R/bench.py --steps 16 --warmup 4
step $O/prof_b8.log timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_b8 -o run -- python3 $R/bench.py --batch-per-gpu 8 --steps 16 --warmup 4
cd $R
for p in prof_b64 prof_b8; do
  nn=$(grep -h ms_per_step $O/$p.log | python -c "import sys,json; r=json.loads(sys.stdin.readline()); print(r['warmup']+r['steps'])")
  python scripts/kstats.py $(ls $O/$p/*/run_results.db $O/$p/run_results.db 2>/dev/null | head -1) --steps $nn --title "$p" --out $O/$p.md || true
done
for f in $O/b*.log $O/f4*.log; do grep -h ms_per_step $f | python -c "
import sys,json
for l in sys.stdin:
    r=json.loads(l); print('$(basename $f)', r['ms_per_step'])
" >> $O/summary.txt || true; done
echo done
