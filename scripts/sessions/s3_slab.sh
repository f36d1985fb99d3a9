set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x -k "slab or linear or ticket or sum" --timeout 120 --timeout-method thread > gpurun_out/s3_slab_tests.log 2>&1
timeout -k 10 200 python bench.py > gpurun_out/s3_slab_bench.log 2>&1
for sp in 8 16 32; do LJS_DW_SPLIT=$sp timeout -k 10 200 python bench.py --steps 30 >> gpurun_out/s3_slab_split.log 2>&1; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof9 -o run -- python bench.py --steps 25 --warmup 5 > gpurun_out/prof9.log 2>&1
