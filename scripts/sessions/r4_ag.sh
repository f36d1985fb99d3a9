# final round-4 build: headline / B=8 / fp8-layer kernel tables, headline PMC passes (MFMA busy),
# the default bench line and 3x driver-shape / B=8 / layer / MSE lines
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r4ag
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then case $rc in 1|2) ;; *) exit $rc;; esac; fi; }
step $O/def.log timeout -k 10 300 python bench.py
for i in 1 2 3; do
step $O/drv_$i.log timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5
step $O/b8_$i.log timeout -k 10 200 python bench.py --batch-per-gpu 8 --steps 20 --warmup 5
done
step $O/layer_bf16.log timeout -k 10 200 python bench.py --model layer --steps 20 --warmup 5
step $O/layer_fp8.log timeout -k 10 200 python bench.py --model layer --fp8 --steps 20 --warmup 5
step $O/mse.log timeout -k 10 200 python bench.py --loss mse --steps 20 --warmup 5
cd /tmp
step $O/prof_b64.log timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_b64 -o run -- python3 $R/bench.py --steps 16 --warmup 4
step $O/prof_b8.log timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_b8 -o run -- python3 $R/bench.py --batch-per-gpu 8 --steps 16 --warmup 4
step $O/prof_l8.log timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_l8 -o run -- python3 $R/bench.py --model layer --fp8 --steps 16 --warmup 4
n=0
for pass in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
            "SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE"; do
  n=$((n+1))
  step $O/pmc_$n.log timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $pass --output-format csv -d $O/pmc_$n -- python3 $R/bench.py --steps 4 --warmup 2 --min-warmup 0 --graph-steps 1
done
cd $R
for p in prof_b64 prof_b8 prof_l8; do
  nn=$(grep -h ms_per_step $O/$p.log | python -c "import sys,json; r=json.loads(sys.stdin.readline()); print(r['warmup']+r['steps'])")
  python scripts/kstats.py $(ls $O/$p/*/run_results.db $O/$p/run_results.db 2>/dev/null | head -1) --steps $nn --title "$p" --out $O/$p.md || true
done
for n in 1 2; do python scripts/pmc_summary.py "$O/pmc_$n/**/*counter_collection.csv" > $O/pmc_$n.txt 2>&1 || true; done
for f in $O/def.log $O/drv_*.log $O/b8_*.log $O/layer_*.log $O/mse.log; do grep -h ms_per_step $f | python -c "
import sys,json
for l in sys.stdin:
    r=json.loads(l); print('$(basename $f)', r['ms_per_step'], r['value'])
" >> $O/summary.txt || true; done
echo done
