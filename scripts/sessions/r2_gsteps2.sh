set -e
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r2gs2.txt
: > $o
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_e2e.py -k "jit_graph" > gpurun_out/r2gs2_test.log 2>&1
for i in 1 2 3; do
  for m in "" "--batch-per-gpu 8"; do
    timeout -k 10 200 python bench.py $m >> $o 2>&1
  done
done
# DP-2 on one GPU over gloo: multi-step capture with segmented graphs
LJS_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 20 --warmup 4 >> $o 2>&1
LJS_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 21 --warmup 3 --graph-steps 1 >> $o 2>&1
