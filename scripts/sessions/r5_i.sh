# lean slab (weight-gradient) GEMM: bit-exact tests and A/B; step lines B=64 / B=8
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r5i
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "lean or slab or gemm_layouts" > $O/tests.log 2>&1 || exit 3
timeout -k 10 300 python scripts/gemm_lean_ab.py > $O/lean.log 2>&1 || exit 3
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/b64_$i.log 2>&1 || exit 3
  LJS_GEMM_LEAN=0 timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/b64_gen_$i.log 2>&1 || exit 3
  timeout -k 10 200 python bench.py --batch-per-gpu 8 --steps 20 --warmup 5 > $O/b8_$i.log 2>&1 || exit 3
  LJS_GEMM_LEAN=0 timeout -k 10 200 python bench.py --batch-per-gpu 8 --steps 20 --warmup 5 > $O/b8_gen_$i.log 2>&1 || exit 3
done
for f in $O/b*.log; do grep -h '^{' $f | python -c "
import sys,json
r=json.loads(sys.stdin.readline()); print('$(basename $f)', r['ms_per_step'])" >> $O/summary.txt; done
echo done
