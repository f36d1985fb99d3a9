# lean GEMM: schedule-pin variant A/B (isolated), then the step with / without the lean kernel and
# with the 256x192 QKV tile, B=64 and B=8 (interleaved x2)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r5g
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "lean or gemm_layouts or tile2562" > $O/tests.log 2>&1 || exit 3
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then case $rc in 1|2) ;; *) exit $rc;; esac; fi; }
V=$R/learning_jax_sharding_amd/_lib/variants/leanpin/libljs_kernels.so
for i in 1 2; do
step $O/var_base_$i.log timeout -k 10 200 python scripts/gemm_lean_var.py
LJS_KERNELS_LIB=$V step $O/var_pin_$i.log timeout -k 10 200 python scripts/gemm_lean_var.py
done
for i in 1 2; do
for cfg in "lean LJS_GEMM_LEAN=1" "gen LJS_GEMM_LEAN=0" "lean2562 LJS_GEMM_TILE2562=1"; do
  set -- $cfg
  env $2 timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/b64_$1_$i.log 2>&1 || exit 3
  env $2 timeout -k 10 200 python bench.py --batch-per-gpu 8 --steps 20 --warmup 5 > $O/b8_$1_$i.log 2>&1 || exit 3
done
done
for i in 1 2; do
  timeout -k 10 120 python scripts/attn_time.py > $O/attn8_$i.log 2>&1 || exit 3
  LJS_ATTN_FWD_RES=16 timeout -k 10 120 python scripts/attn_time.py > $O/attn16_$i.log 2>&1 || exit 3
done
LJS_ATTN_FWD_RES=16 timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/b64_fwd16.log 2>&1 || exit 3
for f in $O/b*_*.log $O/b64_fwd16.log; do grep -h '^{' $f | python -c "
import sys,json
r=json.loads(sys.stdin.readline()); print('$(basename $f)', r['ms_per_step'])" >> $O/summary.txt; done
echo done
