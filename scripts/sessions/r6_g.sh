# round-6: the fused Q/K/V projection + attention forward (correctness, step A/B, trace), and
# where the MX-fp8 up projection's time goes (epilogue ablations + instruction mix)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r6g
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
step $O/tests_k.txt timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "qkv_attn"
step $O/tests_e.txt timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_e2e.py -k "fused_qkv or train_step_matches_eager or multi_step"
for rep in 1 2 3; do
  step $O/b64_on_$rep.txt timeout -k 10 300 python bench.py --steps 20 --warmup 5
  step $O/b64_off_$rep.txt timeout -k 10 300 env LJS_QKV_ATTN=0 python bench.py --steps 20 --warmup 5
done
for rep in 1 2; do
  step $O/b8_on_$rep.txt timeout -k 10 300 python bench.py --batch-per-gpu 8 --steps 20 --warmup 5
  step $O/b8_off_$rep.txt timeout -k 10 300 env LJS_QKV_ATTN=0 python bench.py --batch-per-gpu 8 --steps 20 --warmup 5
done
for f in $O/b*_*.txt; do echo "$(basename $f) $(grep -o '"ms_per_step": [0-9.]*' $f)"; done > $O/lines.txt
cd /tmp
step $O/prof_b64.log timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof_b64 -o run -- python3 $R/bench.py --steps 20 --warmup 5
cd $R
python scripts/kstats.py $O/prof_b64/run_results.db --steps 86 > $O/b64_kernels.md 2>&1
step $O/upproj.txt timeout -k 10 300 python scripts/fp8_upproj_probe.py 20
cd /tmp
step $O/pmc_up.log timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_INSTS_SALU --output-format csv -d $O/pmc_up -- python3 $R/scripts/fp8_upproj_probe.py 3
cd $R
python scripts/pmc_summary.py "$O/pmc_up/**/*counter_collection.csv" > $O/pmc_up.txt 2>&1
echo done
