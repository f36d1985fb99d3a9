set -e
cd "$GRAFT_REPO_ROOT"
R=$PWD
O=$R/gpurun_out/r3ap
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
run() {
  local name=$1; shift; local pass=$1; shift
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $pass --output-format csv -d "$O/$name" -- "$@" > "$O/$name.log" 2>&1
}
P1="SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"
P2="FETCH_SIZE GRBM_GUI_ACTIVE GRBM_COUNT"
P3="SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
P4="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM_RD SQ_INSTS_SMEM SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_INSTS_VALU_TRANS_F32"
for cfg in "64 256 8" "4 4096 8"; do
  tag=$(echo $cfg | tr ' ' '_')
  for w in fwd bwd; do
    run ${w}_${tag}_1 "$P1" python3 $R/scripts/attn_one.py $w $cfg 10
    run ${w}_${tag}_2 "$P2" python3 $R/scripts/attn_one.py $w $cfg 10
    run ${w}_${tag}_3 "$P3" python3 $R/scripts/attn_one.py $w $cfg 10
    run ${w}_${tag}_4 "$P4" python3 $R/scripts/attn_one.py $w $cfg 10
  done
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/kt -o run -- python3 $R/scripts/attn_one.py fwd 64 256 8 20 > $O/kt.log 2>&1
cd "$R"
for d in gpurun_out/r3ap/*/; do python3 scripts/pmc_summary.py "$d**/*counter_collection.csv" > "${d%/}.txt" || true; done
echo done
cd /tmp
for v in 4 8 16 108 116; do
  LJS_ATTN_FWD_RES=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/kt_res$v -o run -- python3 $R/scripts/attn_one.py fwd 64 256 8 20 > $O/kt_res$v.log 2>&1
done
for v in 1 2; do
  LJS_ATTN_FWD_NSUB=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/kt_long_nsub$v -o run -- python3 $R/scripts/attn_one.py fwd 4 4096 8 10 > $O/kt_long_nsub$v.log 2>&1
done
cd "$R"
echo done2
# MX-fp8 FF GEMMs (T=16384): up projection 640 -> 2560 with the fp8 copy, down projection 2560 -> 640
cd /tmp
for cfg in "2560 640 1282 20 qboth" "2560 640 1282 20 qout" "2560 640 1282 20 plain" "640 2560 1282 20 res" "2560 640 2562 20 qboth" "2560 640 1283 20 qboth"; do
  tag=$(echo $cfg | tr ' ' '_')
  timeout -k 10 120 python3 $R/scripts/fp8_one.py $cfg > $O/f8_$tag.time 2>&1
done
run f8_up_1 "$P1" python3 $R/scripts/fp8_one.py 2560 640 1282 10 qboth
run f8_up_2 "$P2" python3 $R/scripts/fp8_one.py 2560 640 1282 10 qboth
run f8_up_3 "$P3" python3 $R/scripts/fp8_one.py 2560 640 1282 10 qboth
run f8_up_4 "$P4" python3 $R/scripts/fp8_one.py 2560 640 1282 10 qboth
cd "$R"
for d in gpurun_out/r3ap/f8*/; do python3 scripts/pmc_summary.py "$d**/*counter_collection.csv" > "${d%/}.txt" || true; done
echo done3
