# f32 residual rounded to bf16 before its 2-D all-to-all; weight shadows cast straight into their
# buffers: full GPU suite, smoke, 2-D layer (bf16 / MX-fp8) and block rehearsals, 1x1 lines,
# 2-D bf16 and MX-fp8 layer tables
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r4af
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then case $rc in 1|2) ;; *) exit $rc;; esac; fi; }
step $O/gpu_tests.log timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/
if grep -q " failed\|[0-9] error" $O/gpu_tests.log; then echo "tests failed"; tail -40 $O/gpu_tests.log; exit 1; fi
step $O/smoke.log timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()"
F4="WORLD_SIZE=4 RANK=0 LOCAL_RANK=0 LJS_DIST_BACKEND=fake MASTER_ADDR=127.0.0.1"
for i in 1 2; do
step $O/f4_2d_l8_$i.log env $F4 MASTER_PORT=2994$i timeout -k 10 200 python bench.py --gpus 4 --mesh 2d --model layer --fp8 --steps 20 --warmup 5
step $O/f4_2d_l_$i.log env $F4 MASTER_PORT=2995$i timeout -k 10 200 python bench.py --gpus 4 --mesh 2d --model layer --steps 20 --warmup 5
step $O/l8_$i.log timeout -k 10 200 python bench.py --model layer --fp8 --steps 20 --warmup 5
step $O/drv_$i.log timeout -k 10 200 python bench.py --steps 20 --warmup 5
step $O/f4_2d_$i.log env $F4 MASTER_PORT=2997$i timeout -k 10 200 python bench.py --gpus 4 --mesh 2d --steps 20 --warmup 5
step $O/b8_$i.log timeout -k 10 200 python bench.py --batch-per-gpu 8 --steps 20 --warmup 5
done
step $O/trace_2d_fp8.log env $F4 MASTER_PORT=29961 LJS_ATEN_TRACE=$O/aten_2d_l.txt timeout -k 10 300 python bench.py --gpus 4 --mesh 2d --model layer --steps 2 --warmup 2 --min-warmup 0
cd /tmp
export WORLD_SIZE=4 RANK=0 LOCAL_RANK=0 LJS_DIST_BACKEND=fake MASTER_ADDR=127.0.0.1
step $O/prof_2d_l.log env MASTER_PORT=29962 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_2d_l -o run -- python3 $R/bench.py --gpus 4 --mesh 2d --model layer --steps 16 --warmup 4
step $O/prof_2d_l8.log env MASTER_PORT=29963 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_2d_l8 -o run -- python3 $R/bench.py --gpus 4 --mesh 2d --model layer --fp8 --steps 16 --warmup 4
cd $R
for p in prof_2d_l prof_2d_l8; do
  nn=$(grep -h ms_per_step $O/$p.log | python -c "import sys,json; r=json.loads(sys.stdin.readline()); print(r['warmup']+r['steps'])")
  python scripts/kstats.py $(ls $O/$p/*/run_results.db $O/$p/run_results.db 2>/dev/null | head -1) --steps $nn --title "$p" --out $O/$p.md || true
done
for f in $O/f4_*.log $O/l8*.log $O/drv*.log $O/b8*.log $O/prof_*.log; do grep -h ms_per_step $f | python -c "
import sys,json
for l in sys.stdin:
    r=json.loads(l); print('$(basename $f)', r['ms_per_step'], r['value'])
" >> $O/summary.txt || true; done
echo done
