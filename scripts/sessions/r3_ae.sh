cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r3ae
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; if [ $rc -ne 0 ]; then echo "rc=$rc: $*" >> $O/rc.log; case $rc in 1|2) ;; *) exit $rc;; esac; fi; }
F4="WORLD_SIZE=4 RANK=0 LOCAL_RANK=0 LJS_DIST_BACKEND=fake MASTER_ADDR=127.0.0.1"
step $O/fake4_2d.log env $F4 MASTER_PORT=29671 timeout -k 10 300 python bench.py --gpus 4 --mesh 2d
step $O/fake4_dp.log env $F4 MASTER_PORT=29672 timeout -k 10 300 python bench.py --gpus 4 --mesh dp
step $O/fake8_dp.log env WORLD_SIZE=8 RANK=0 LOCAL_RANK=0 LJS_DIST_BACKEND=fake MASTER_ADDR=127.0.0.1 MASTER_PORT=29673 timeout -k 10 300 python bench.py --gpus 8 --mesh dp
step $O/v2x2.log env LJS_NUM_DEVICES=4 timeout -k 10 300 python bench.py --mesh 2x2
step $O/fsdp4.log env LJS_NUM_DEVICES=4 timeout -k 10 300 python bench.py --model fsdp --mesh 4x1
step $O/case5.log env LJS_NUM_DEVICES=4 timeout -k 10 300 python bench.py --mesh 4x1 --rules case5
step $O/ff.log timeout -k 10 200 python bench.py --model ff
step $O/ff8.log timeout -k 10 200 python bench.py --model ff --fp8
step $O/seq1k.log timeout -k 10 200 python bench.py --seq 1024 --batch-per-gpu 16
step $O/ring.log timeout -k 10 300 python scripts/ring_trace.py
echo done
