# MX-fp8 FF block in the activation's storage row order + the seq-major out projection's residual
# transposed/rounded by one pass (no torch clones in the 2-D layer step): full GPU suite, 2-D
# MX-fp8 layer rehearsal lines + table, 1x1 fp8 layer and headline lines
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r4ad
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then case $rc in 1|2) ;; *) exit $rc;; esac; fi; }
step $O/gpu_tests.log timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/
if grep -q " failed\|[0-9] error" $O/gpu_tests.log; then echo "tests failed"; tail -40 $O/gpu_tests.log; exit 1; fi
F4="WORLD_SIZE=4 RANK=0 LOCAL_RANK=0 LJS_DIST_BACKEND=fake MASTER_ADDR=127.0.0.1"
for i in 1 2; do
step $O/f4_2d_l8_$i.log env $F4 MASTER_PORT=2994$i timeout -k 10 200 python bench.py --gpus 4 --mesh 2d --model layer --fp8 --steps 20 --warmup 5
step $O/f4_2d_l_$i.log env $F4 MASTER_PORT=2995$i timeout -k 10 200 python bench.py --gpus 4 --mesh 2d --model layer --steps 20 --warmup 5
step $O/l8_$i.log timeout -k 10 200 python bench.py --model layer --fp8 --steps 20 --warmup 5
step $O/drv_$i.log timeout -k 10 200 python bench.py --steps 20 --warmup 5
done
step $O/trace_2d_fp8.log env $F4 MASTER_PORT=29961 LJS_ATEN_TRACE=$O/aten_2d_fp8.txt timeout -k 10 300 python bench.py --gpus 4 --mesh 2d --model layer --fp8 --steps 2 --warmup 2 --min-warmup 0
cd /tmp
export WORLD_SIZE=4 RANK=0 LOCAL_RANK=0 LJS_DIST_BACKEND=fake MASTER_ADDR=127.0.0.1
step $O/prof_2d_fp8.log env MASTER_PORT=29962 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_2d_fp8 -o run -- python3 $R/bench.py --gpus 4 --mesh 2d --model layer --fp8 --steps 16 --warmup 4
cd $R
for p in prof_2d_fp8; do
  nn=$(grep -h ms_per_step $O/$p.log | python -c "import sys,json; r=json.loads(sys.stdin.readline()); print(r['warmup']+r['steps'])")
  python scripts/kstats.py $(ls $O/$p/*/run_results.db $O/$p/run_results.db 2>/dev/null | head -1) --steps $nn --title "$p" --out $O/$p.md || true
done
for f in $O/f4_*.log $O/l8*.log $O/drv*.log $O/prof_*.log; do grep -h ms_per_step $f | python -c "
import sys,json
for l in sys.stdin:
    r=json.loads(l); print('$(basename $f)', r['ms_per_step'], r['value'])
" >> $O/summary.txt || true; done
echo done
