#!/bin/bash
# Deeper counter passes for single GEMM configs: scripts/pmc_gemm2.sh OUTDIR "case tile sk" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
out=$1; shift; mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
i=0
for cfg in "$@"; do
  i=$((i+1))
  n=0
  for pass in "SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INST_CYCLES_VMEM_RD SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" \
              "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE" \
              "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TA_BUSY_avr TCC_EA0_RDREQ_DRAM_sum"; do
    n=$((n+1))
    timeout -k 10 120 rocprofv3 --kernel-trace --pmc $pass --output-format csv -d "$R/$out/c${i}_$n" -- python3 "$R/scripts/gemm_one.py" $cfg 20 > "$R/$out/c${i}_$n.log" 2>&1 || exit $?
  done
  echo "== $cfg"
  for n in 1 2 3; do python3 "$R/scripts/pmc_summary.py" "$R/$out/c${i}_$n/**/*counter_collection.csv" | grep -A10 "gemm_dma" | grep -v "^##"; done
done
