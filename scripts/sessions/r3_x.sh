cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r3x
mkdir -p $O
i=0
for pass in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
            "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE" \
            "SQ_WAIT_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU"; do
  i=$((i+1))
  for cfg in "640 2560 256160 10 res" "2560 640 1282 10 qboth"; do
    tag=$(echo $cfg | tr ' ' '_')
    timeout -s KILL 90 rocprofv3 --pmc $pass --output-format csv -d $O/p${i}_$tag -- python scripts/fp8_one.py $cfg > $O/p${i}_$tag.log 2>&1 || { echo "pass $i $cfg rc=$?"; exit 1; }
  done
done
for i in 1 2 3; do for tag in 640_2560_256160_10_res 2560_640_1282_10_qboth; do echo "== pass $i $tag"; python scripts/pmc_summary.py "$O/p${i}_$tag/**/*counter_collection.csv"; done; done > $O/summary.txt 2>&1
echo done
