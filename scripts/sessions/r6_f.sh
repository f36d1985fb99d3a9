# round-6: where the MX-fp8 up projection's 61 us go (epilogue ablations + instruction mix)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r6f
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
step $O/upproj.txt timeout -k 10 300 python scripts/fp8_upproj_probe.py 20
cd /tmp
step $O/pmc_up.log timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_INSTS_SALU --output-format csv -d $O/pmc_up -- python3 $R/scripts/fp8_upproj_probe.py 3
cd $R
python scripts/pmc_summary.py "$O/pmc_up/**/*counter_collection.csv" > $O/pmc_up.txt 2>&1
echo done
