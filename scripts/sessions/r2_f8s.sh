set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k "fp8" > gpurun_out/r2fs_tests.log 2>&1
o=gpurun_out/r2fs.txt
: > $o
for t in 1282 2563; do
  for m in qout qmask; do timeout -k 10 60 python scripts/fp8_one.py 2560 640 $t 50 $m 2>&1 | grep -v amdgpu.ids >> $o; done
  for m in plain res; do timeout -k 10 60 python scripts/fp8_one.py 640 2560 $t 50 $m 2>&1 | grep -v amdgpu.ids >> $o; done
done
for i in 1 2; do
echo "fp8 layer $(timeout -k 10 200 python bench.py --steps 100 --warmup 20 --model layer --fp8 2>&1 | grep -o '"ms_per_step": [0-9.]*')" >> $o
echo "bf16 layer $(timeout -k 10 200 python bench.py --steps 100 --warmup 20 --model layer 2>&1 | grep -o '"ms_per_step": [0-9.]*')" >> $o
done
