cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r3z
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; if [ $rc -ne 0 ]; then echo "rc=$rc: $*" >> $O/rc.log; case $rc in 1|2) ;; *) exit $rc;; esac; fi; }
F4="WORLD_SIZE=4 RANK=0 LOCAL_RANK=0 LJS_DIST_BACKEND=fake MASTER_ADDR=127.0.0.1"
step $O/b64.log timeout -k 10 200 python bench.py
step $O/b64_2.log timeout -k 10 200 python bench.py
step $O/b8.log timeout -k 10 200 python bench.py --batch-per-gpu 8
step $O/mse.log timeout -k 10 200 python bench.py --loss mse
step $O/layer.log timeout -k 10 200 python bench.py --model layer
step $O/layer8.log timeout -k 10 200 python bench.py --model layer --fp8
step $O/ff.log timeout -k 10 200 python bench.py --model ff
step $O/ff8.log timeout -k 10 200 python bench.py --model ff --fp8
step $O/long.log timeout -k 10 200 python bench.py --seq 4096 --batch-per-gpu 4
step $O/fsdp4.log env LJS_NUM_DEVICES=4 timeout -k 10 300 python bench.py --model fsdp
step $O/case5_4.log env LJS_NUM_DEVICES=4 timeout -k 10 300 python bench.py --mesh 4x1 --rules case5
step $O/v2x2.log env LJS_NUM_DEVICES=4 timeout -k 10 300 python bench.py --mesh 2x2
step $O/fake4_2d.log env $F4 MASTER_PORT=29671 timeout -k 10 300 python bench.py --gpus 4 --mesh 2d
step $O/fake4_dp.log env $F4 MASTER_PORT=29672 timeout -k 10 300 python bench.py --gpus 4 --mesh dp
step $O/ring.log timeout -k 10 200 python scripts/ring_trace.py
cd /tmp
step $O/prof_b64.log timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_b64 -o run -- python3 $R/bench.py --steps 24 --warmup 6
step $O/prof_b8.log timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_b8 -o run -- python3 $R/bench.py --batch-per-gpu 8 --steps 24 --warmup 6
echo done
