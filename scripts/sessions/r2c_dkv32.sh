set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -q -x -k "attention or attn" --timeout 120 --timeout-method thread > gpurun_out/r2c_dkv32_tests.log 2>&1
out=gpurun_out/r2c_dkv32.log
for rep in 1 2; do
for cfg in "LJS_ATTN_DKV32=0" "LJS_ATTN_DQ32=0" "LJS_ATTN_DQ32=1"; do
  for a in "--seq 4096 --batch-per-gpu 4" "--seq 1024 --batch-per-gpu 16"; do
    r=$(env $cfg timeout -k 10 120 python bench.py --steps 24 --warmup 8 $a | tail -1 | python -c "import json,sys; print(json.loads(sys.stdin.read())['ms_per_step'])")
    echo "$cfg [$a] $r" >> $out
  done
done
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r2c_dkv32_4k -o prof -- python bench.py --steps 16 --warmup 8 --seq 4096 --batch-per-gpu 4 > /dev/null 2>&1
