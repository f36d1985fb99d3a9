set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 100 python scripts/small_kernels.py > gpurun_out/s3_small.log 2>&1
for nb in 64 128 512 1024; do LJS_SUM_BLOCKS=$nb timeout -k 10 60 python scripts/small_kernels.py sum | sed "s/^/blocks=$nb /" >> gpurun_out/s3_small.log 2>&1; done
