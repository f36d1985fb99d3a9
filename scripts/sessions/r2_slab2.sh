set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for i in 1 2; do
for cfg in "LJS_GEMM_ORDER=1 LJS_DW_SLAB_MODE=1" "LJS_GEMM_ORDER=0 LJS_DW_SLAB_MODE=1" "LJS_GEMM_ORDER=0 LJS_DW_SLAB_MODE=0"; do
  for b in 64 8; do
    env $cfg timeout -k 10 200 python bench.py --steps 100 --warmup 20 --batch-per-gpu $b > gpurun_out/r2s2.log 2>&1
    echo "$cfg b=$b $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r2s2.log)" >> gpurun_out/r2s2_ab.txt
  done
done
done
