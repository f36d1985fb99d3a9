# clock-ramp A/B (scratch-GEMM ramp instead of extra warmup steps); GEMM fragment-pin A/B
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r4m
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then case $rc in 1|2) ;; *) exit $rc;; esac; fi; }
NOPIN=$R/learning_jax_sharding_amd/_lib/variants/nopin/libljs_kernels.so
step $O/smoke.log timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()"
step $O/tests.log timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemm or slab"
for i in 1 2; do
step $O/gemm_pin_$i.log timeout -k 10 200 python scripts/gemm_ab.py
step $O/gemm_nopin_$i.log env LJS_KERNELS_LIB=$NOPIN timeout -k 10 200 python scripts/gemm_ab.py
done
for i in 1 2; do
step $O/warm64_$i.log timeout -k 10 200 python bench.py --steps 20 --warmup 5
step $O/nopin64_$i.log env LJS_KERNELS_LIB=$NOPIN timeout -k 10 200 python bench.py --steps 20 --warmup 5
step $O/ramp30_$i.log timeout -k 10 200 python bench.py --steps 20 --warmup 5 --min-warmup 0 --clock-ramp-ms 30
step $O/ramp100_$i.log timeout -k 10 200 python bench.py --steps 20 --warmup 5 --min-warmup 0 --clock-ramp-ms 100
step $O/none_$i.log timeout -k 10 200 python bench.py --steps 20 --warmup 5 --min-warmup 0
done
step $O/b8_ramp100.log timeout -k 10 200 python bench.py --batch-per-gpu 8 --steps 20 --warmup 5 --min-warmup 0 --clock-ramp-ms 100
step $O/b8_warm64.log timeout -k 10 200 python bench.py --batch-per-gpu 8 --steps 20 --warmup 5
for f in $O/*.log; do grep -h ms_per_step $f | python -c "
import sys,json
for l in sys.stdin:
    r=json.loads(l); c=r['config']; print('$(basename $f)', r['ms_per_step'], r['warmup'], c.get('clock_ramp_ms'), c['global_batch'])
" >> $O/summary.txt || true; done
echo done
