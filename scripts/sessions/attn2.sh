set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x -k "attention" --timeout 120 --timeout-method thread > gpurun_out/attn2_tests.log 2>&1
for n in 1 2; do LJS_ATTN_FWD_NSUB=$n timeout -k 10 100 python scripts/attn_bench.py > gpurun_out/attn2_n$n.log 2>&1; done
timeout -k 10 200 python bench.py > gpurun_out/bench_attn2.log 2>&1
