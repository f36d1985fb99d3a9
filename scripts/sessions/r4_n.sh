# Adam heavy-first A/B; slab-traffic weight sweep (fewer dW slabs: cheaper Adam, longer dW GEMM);
# kernel tables of the current build at B=64 / B=8
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r4n
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then case $rc in 1|2) ;; *) exit $rc;; esac; fi; }
for i in 1 2; do
for B in 64 8; do
step $O/b${B}_hf1_$i.log timeout -k 10 200 python bench.py --batch-per-gpu $B --steps 20 --warmup 5
step $O/b${B}_hf0_$i.log env LJS_ADAM_HEAVY_FIRST=0 timeout -k 10 200 python bench.py --batch-per-gpu $B --steps 20 --warmup 5
step $O/b${B}_tw2_$i.log env LJS_DW_TRAFFIC_W=2 timeout -k 10 200 python bench.py --batch-per-gpu $B --steps 20 --warmup 5
step $O/b${B}_tw4_$i.log env LJS_DW_TRAFFIC_W=4 timeout -k 10 200 python bench.py --batch-per-gpu $B --steps 20 --warmup 5
done
done
cd /tmp
step $O/prof_b64.log timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_b64 -o run -- python3 $R/bench.py --steps 16 --warmup 4
step $O/prof_b64_hf0.log env LJS_ADAM_HEAVY_FIRST=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_b64_hf0 -o run -- python3 $R/bench.py --steps 16 --warmup 4
step $O/prof_b8.log timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_b8 -o run -- python3 $R/bench.py --batch-per-gpu 8 --steps 16 --warmup 4
cd $R
for p in prof_b64 prof_b64_hf0 prof_b8; do
  n=$(grep -h ms_per_step $O/$p.log | python -c "import sys,json; r=json.loads(sys.stdin.readline()); print(r['warmup']+r['steps'])")
  python scripts/kstats.py $(ls $O/$p/*/run_results.db $O/$p/run_results.db 2>/dev/null | head -1) --steps $n --title "$p" --out $O/$p.md || true
done
for f in $O/b*.log; do grep -h ms_per_step $f | python -c "
import sys,json
for l in sys.stdin:
    r=json.loads(l); print('$(basename $f)', r['ms_per_step'])
" >> $O/summary.txt || true; done
echo done
