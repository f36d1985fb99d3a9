# round-4 final build: the secondary configurations of the README table (long context, FF, FSDP,
# case5 rules, virtual-device and fake-rank rehearsals), two runs each
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r4aa
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then case $rc in 1|2) ;; *) exit $rc;; esac; fi; }
F4="WORLD_SIZE=4 RANK=0 LOCAL_RANK=0 LJS_DIST_BACKEND=fake MASTER_ADDR=127.0.0.1"
for i in 1 2; do
step $O/s4096_$i.log timeout -k 10 300 python bench.py --seq 4096 --batch-per-gpu 4 --steps 20 --warmup 5
step $O/s1024_$i.log timeout -k 10 300 python bench.py --seq 1024 --batch-per-gpu 16 --steps 20 --warmup 5
step $O/ff_$i.log timeout -k 10 300 python bench.py --model ff --steps 20 --warmup 5
step $O/ff8_$i.log timeout -k 10 300 python bench.py --model ff --fp8 --steps 20 --warmup 5
step $O/fsdp4v_$i.log env LJS_NUM_DEVICES=4 timeout -k 10 300 python bench.py --model fsdp --mesh 4x1 --steps 20 --warmup 5
step $O/case5v_$i.log env LJS_NUM_DEVICES=4 timeout -k 10 300 python bench.py --mesh 4x1 --rules case5 --steps 20 --warmup 5
step $O/v2x2_$i.log env LJS_NUM_DEVICES=4 timeout -k 10 300 python bench.py --mesh 2x2 --steps 20 --warmup 5
step $O/f4_2d_$i.log env $F4 MASTER_PORT=2986$i timeout -k 10 300 python bench.py --gpus 4 --mesh 2d --steps 20 --warmup 5
step $O/f4_dp_$i.log env $F4 MASTER_PORT=2987$i timeout -k 10 300 python bench.py --gpus 4 --mesh dp --steps 20 --warmup 5
step $O/f4_2d_l8_$i.log env $F4 MASTER_PORT=2988$i timeout -k 10 300 python bench.py --gpus 4 --mesh 2d --model layer --fp8 --steps 20 --warmup 5
done
step $O/fsdp4096.log timeout -k 10 300 python bench.py --model fsdp --dim 4096 --steps 10 --warmup 3
for f in $O/*.log; do grep -h ms_per_step $f | python -c "
import sys,json
for l in sys.stdin:
    r=json.loads(l); print('$(basename $f)', r['ms_per_step'], r['value'], r['config']['parallelism'])
" >> $O/summary.txt || true; done
echo done
