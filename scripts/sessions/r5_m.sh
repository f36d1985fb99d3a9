# conflict-free dS^T image in the fused attention backward; Adam with 256 / 512 / 1024 threads per
# 64x64 tile (LJS_ADAM_THREADS): attention + Adam GPU tests, then step kernel tables
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r5m
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
step $O/tests.log timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu -k "attn or attention or adam or flash or sdpa" tests/test_kernels_gpu.py tests/test_gpu_e2e.py
cd /tmp
for cfg in "b64 256 64" "b64t1024 1024 64" "b64t512 512 64" "b8 256 8" "b8t1024 1024 8"; do
  set -- $cfg
  LJS_ADAM_THREADS=$2 step $O/prof_$1.log timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$1 -o run -- python3 $R/bench.py --batch-per-gpu $3 --steps 16 --warmup 4
done
cd $R
for p in b64 b64t1024 b64t512 b8 b8t1024; do
  nn=$(grep -h ms_per_step $O/prof_$p.log | python -c "import sys,json; r=json.loads(sys.stdin.readline()); print(r['warmup']+r['steps'])")
  python scripts/kstats.py $(ls $O/prof_$p/*/run_results.db $O/prof_$p/run_results.db 2>/dev/null | head -1) --steps $nn --title "$p" --out $O/prof_$p.md > /dev/null 2>&1 || true
done
echo done
