set -e
cd "$GRAFT_REPO_ROOT"
R=$PWD
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_gpu_e2e.py -q -x -k "attention or attn or ring" --timeout 120 --timeout-method thread > gpurun_out/r2c_fin2_tests.log 2>&1
out=gpurun_out/r2c_fin2.log
for rep in 1 2; do
  for a in "--seq 4096 --batch-per-gpu 4" "--batch-per-gpu 8"; do
    r=$(timeout -k 10 120 python bench.py --steps 48 --warmup 8 $a | tail -1 | python -c "import json,sys; print(json.loads(sys.stdin.read())['ms_per_step'])")
    echo "[$a] $r" >> $out
  done
done
mkdir -p gpurun_out/r2c_pmc32b
cd /tmp
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT \
  --output-format csv -d $R/gpurun_out/r2c_pmc32b/a1 -- python3 $R/scripts/attn_one.py bwd 4 4096 8 6 > $R/gpurun_out/r2c_pmc32b/a1.log 2>&1
