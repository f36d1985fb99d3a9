# (r5aw: re-run of r5_l.sh on the current build) fake-4 rehearsal (rank 0 of 4; collectives move nothing): dp vs 2-D bf16 block, 2-D MX-fp8 layer --
# lines and kernel tables with the round-5 build
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r5aw
mkdir -p $O
F4="WORLD_SIZE=4 RANK=0 LOCAL_RANK=0 LJS_DIST_BACKEND=fake MASTER_ADDR=127.0.0.1"
for i in 1 2; do
  env $F4 MASTER_PORT=2991$i timeout -k 10 200 python bench.py --gpus 4 --mesh 2d --steps 20 --warmup 5 > $O/f4_2d_$i.log 2>&1 || exit 3
  env $F4 MASTER_PORT=2992$i timeout -k 10 200 python bench.py --gpus 4 --mesh dp --secondary off --steps 20 --warmup 5 > $O/f4_dp_$i.log 2>&1 || exit 3
done
cd /tmp
env $F4 MASTER_PORT=29931 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_2d -o run -- python3 $R/bench.py --gpus 4 --mesh 2d --steps 16 --warmup 4 > $O/prof_2d.log 2>&1 || exit 3
env $F4 MASTER_PORT=29932 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_dp -o run -- python3 $R/bench.py --gpus 4 --mesh dp --secondary off --steps 16 --warmup 4 > $O/prof_dp.log 2>&1 || exit 3
env $F4 MASTER_PORT=29933 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_2d_fp8 -o run -- python3 $R/bench.py --gpus 4 --mesh 2d --model layer --fp8 --steps 16 --warmup 4 > $O/prof_2d_fp8.log 2>&1 || exit 3
cd $R
for p in prof_2d prof_dp prof_2d_fp8; do
  nn=$(grep -h ms_per_step $O/$p.log | python -c "import sys,json; r=json.loads(sys.stdin.readline()); print(r['warmup']+r['steps'])")
  python scripts/kstats.py $(ls $O/$p/*/run_results.db $O/$p/run_results.db 2>/dev/null | head -1) --steps $nn --title "$p" --out $O/$p.md > /dev/null 2>&1 || true
done
for f in $O/f4_*.log $O/prof_*.log; do grep -h ms_per_step $f | python -c "
import sys,json
for l in sys.stdin:
    r=json.loads(l); print('$(basename $f)', r['ms_per_step'], r['value'])
" >> $O/summary.txt || true; done
echo done
