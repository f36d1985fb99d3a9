# bf16 slabs: per-kernel deltas at B=64 / B=8; the 2-D replay's input copies
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r4k
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then case $rc in 1|2) ;; *) exit $rc;; esac; fi; }
F4="WORLD_SIZE=4 RANK=0 LOCAL_RANK=0 LJS_DIST_BACKEND=fake MASTER_ADDR=127.0.0.1"
step $O/replay_2d.log env $F4 MASTER_PORT=29731 LJS_REPLAY_TRACE=1 timeout -k 10 300 python bench.py --gpus 4 --mesh 2d --steps 20 --warmup 5
cd /tmp
step $O/prof_b64_s16.log env LJS_SLAB_BF16=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_b64_s16 -o run -- python3 $R/bench.py --steps 16 --warmup 4
step $O/prof_b8_s16.log env LJS_SLAB_BF16=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_b8_s16 -o run -- python3 $R/bench.py --batch-per-gpu 8 --steps 16 --warmup 4
step $O/prof_b8.log timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_b8 -o run -- python3 $R/bench.py --batch-per-gpu 8 --steps 16 --warmup 4
cd $R
for i in 1 2; do
step $O/b64_$i.log timeout -k 10 200 python bench.py --steps 20 --warmup 5
step $O/b64_s16_$i.log env LJS_SLAB_BF16=1 timeout -k 10 200 python bench.py --steps 20 --warmup 5
step $O/b8_$i.log timeout -k 10 200 python bench.py --batch-per-gpu 8 --steps 20 --warmup 5
step $O/b8_s16_$i.log env LJS_SLAB_BF16=1 timeout -k 10 200 python bench.py --batch-per-gpu 8 --steps 20 --warmup 5
done
echo done
