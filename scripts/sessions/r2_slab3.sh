set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for m in 1 0; do
LJS_DW_SLAB_MODE=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r2s3_prof$m -o prof -- python bench.py --steps 20 --warmup 5 > gpurun_out/r2s3_prof$m.log 2>&1
done
