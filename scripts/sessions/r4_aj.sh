# MX-fp8 FF weight-gradient split count A/B (LJS_MX_WGRAD_SPLIT_MAX): fewer f32 slabs for Adam to
# read vs fewer workgroups in the weight-gradient GEMM; fp8 layer lines x3 interleaved + tables
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r4aj
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then case $rc in 1|2) ;; *) exit $rc;; esac; fi; }
for i in 1 2 3; do
for sm in 64 4 3 2; do
step $O/l8_s${sm}_$i.log env LJS_MX_WGRAD_SPLIT_MAX=$sm timeout -k 10 200 python bench.py --model layer --fp8 --steps 20 --warmup 5
done
done
cd /tmp
for sm in 64 3; do
step $O/prof_s$sm.log env LJS_MX_WGRAD_SPLIT_MAX=$sm timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_s$sm -o run -- python3 $R/bench.py --model layer --fp8 --steps 16 --warmup 4
done
cd $R
for p in prof_s64 prof_s3; do
  nn=$(grep -h ms_per_step $O/$p.log | python -c "import sys,json; r=json.loads(sys.stdin.readline()); print(r['warmup']+r['steps'])")
  python scripts/kstats.py $(ls $O/$p/*/run_results.db $O/$p/run_results.db 2>/dev/null | head -1) --steps $nn --title "$p" --out $O/$p.md || true
done
for f in $O/l8*.log; do grep -h ms_per_step $f | python -c "
import sys,json
for l in sys.stdin:
    r=json.loads(l); print('$(basename $f)', r['ms_per_step'], r['value'])
" >> $O/summary.txt || true; done
echo done
