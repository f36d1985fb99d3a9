set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_epilogue_gpu.py -x -q --timeout 200 --timeout-method thread -k "fp8 or ff_block or side_stream" > gpurun_out/r2v4_tests.log 2>&1
o=gpurun_out/r2v4.txt
: > $o
for i in 1 2; do
echo "fp8 layer $(timeout -k 10 200 python bench.py --steps 100 --warmup 20 --model layer --fp8 2>&1 | grep -o '"ms_per_step": [0-9.]*')" >> $o
echo "bf16 layer $(timeout -k 10 200 python bench.py --steps 100 --warmup 20 --model layer 2>&1 | grep -o '"ms_per_step": [0-9.]*')" >> $o
echo "fp8 ff $(timeout -k 10 200 python bench.py --steps 100 --warmup 20 --model ff --fp8 2>&1 | grep -o '"ms_per_step": [0-9.]*')" >> $o
echo "bf16 ff $(timeout -k 10 200 python bench.py --steps 100 --warmup 20 --model ff 2>&1 | grep -o '"ms_per_step": [0-9.]*')" >> $o
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r2v4_prof -o prof -- python bench.py --steps 20 --warmup 5 --model layer --fp8 > gpurun_out/r2v4_prof.log 2>&1
