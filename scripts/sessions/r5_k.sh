# two-sub-tile attention forward: bit-exact test, isolated timing, step A/B (B=64, B=8)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r5k
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "two_subtiles or vst_bit_exact or attention_fwd_bwd" > $O/tests.log 2>&1 || exit 3
for i in 1 2; do
  for v in 0 4 8; do
    LJS_ATTN_FWD_RES2=$v timeout -k 10 120 python scripts/attn_time.py > $O/attn_${v}_$i.log 2>&1 || exit 3
  done
done
for i in 1 2; do
  for v in 0 4 8; do
    LJS_ATTN_FWD_RES2=$v timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/b64_${v}_$i.log 2>&1 || exit 3
  done
  for v in 0 4; do
    LJS_ATTN_FWD_RES2=$v timeout -k 10 200 python bench.py --batch-per-gpu 8 --steps 20 --warmup 5 > $O/b8_${v}_$i.log 2>&1 || exit 3
  done
done
for f in $O/b*.log; do grep -h '^{' $f | python -c "
import sys,json
r=json.loads(sys.stdin.readline()); print('$(basename $f)', r['ms_per_step'])" >> $O/summary.txt; done
echo done
