#!/bin/bash
# Counter runs for single GEMM configs: scripts/pmc_gemm.sh OUTDIR "case tile sk" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
out=$1; shift; mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
i=0
for cfg in "$@"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT \
    --output-format csv -d "$R/$out/c$i" -- python3 "$R/scripts/gemm_one.py" $cfg 20 > "$R/$out/c$i.log" 2>&1 || exit $?
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc TA_BUSY_avr TCP_TOTAL_CACHE_ACCESSES_sum SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM \
    --output-format csv -d "$R/$out/d$i" -- python3 "$R/scripts/gemm_one.py" $cfg 20 > "$R/$out/d$i.log" 2>&1 || exit $?
  echo "== $cfg"; python3 "$R/scripts/pmc_summary.py" "$R/$out/c$i/**/*counter_collection.csv" | grep -A12 gemm
  python3 "$R/scripts/pmc_summary.py" "$R/$out/d$i/**/*counter_collection.csv" | grep -A12 gemm
done
