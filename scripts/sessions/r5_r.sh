# (1) weight-gradient GEMMs as 8-wave 4-stage 128x128 blocks at one round (LJS_DW_BIG_TILE=12884:
#     dW_qkv 4 splits, dW_o 12 -- half the slab bytes Adam reads) vs the 2-block 1282 tiles
#     (8 / 24 splits), interleaved x2 at B=64, plus the 12884 two-round form; (2) steps x graph size
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r5r
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
# kernel arguments in device memory (HIP_FORCE_DEV_KERNARG=1) vs the runtime default: every
# kernel's first scalar loads read its arguments
step $O/probe_kdefault.txt timeout -k 10 120 python scripts/adam_probe.py
HIP_FORCE_DEV_KERNARG=1 step $O/probe_kdev.txt timeout -k 10 120 python scripts/adam_probe.py
HIP_FORCE_DEV_KERNARG=0 step $O/probe_khost.txt timeout -k 10 120 python scripts/adam_probe.py
for rep in 1 2; do
  HIP_FORCE_DEV_KERNARG=1 step $O/b64_kdev_$rep.txt timeout -k 10 300 python bench.py
  HIP_FORCE_DEV_KERNARG=1 step $O/b8_kdev_$rep.txt timeout -k 10 300 python bench.py --batch-per-gpu 8
  step $O/b8_default_$rep.txt timeout -k 10 300 python bench.py --batch-per-gpu 8
done
for rep in 1 2; do
  step $O/b64_1282_$rep.txt timeout -k 10 300 python bench.py
  LJS_DW_BIG_TILE=12884 step $O/b64_12884_$rep.txt timeout -k 10 300 python bench.py
  LJS_DW_BIG_TILE=12884 LJS_DW_BIG_ROUNDS=2 step $O/b64_12884r2_$rep.txt timeout -k 10 300 python bench.py
done
cd /tmp
LJS_DW_BIG_TILE=12884 step $O/prof_12884.log timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_12884 -o run -- python3 $R/bench.py --steps 16 --warmup 4
cd $R
nn=$(grep -h ms_per_step $O/prof_12884.log | python -c "import sys,json; r=json.loads(sys.stdin.readline()); print(r['warmup']+r['steps'])")
python scripts/kstats.py $(ls $O/prof_12884/*/run_results.db $O/prof_12884/run_results.db 2>/dev/null | head -1) --steps $nn --title 12884 --out $O/prof_12884.md > /dev/null 2>&1 || true
for cfg in "40 5" "40 20" "40 40" "20 20" "20 5" "80 20"; do
  set -- $cfg
  step $O/s$1_g$2.txt timeout -k 10 300 python bench.py --steps $1 --warmup 5 --graph-steps $2
done
echo done
