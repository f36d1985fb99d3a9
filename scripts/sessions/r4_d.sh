# Adam tile-size A/B (B=64, B=8), the B=8 kernel table, the fp8 layer (1x1 and the fake-4 2-D
# rehearsal with its kernel table), the bf16 fake-4 2-D table
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r4d
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then case $rc in 1|2) ;; *) exit $rc;; esac; fi; }
for rows in 64 32 16; do
  step $O/b64_rows$rows.log env LJS_ADAM_ROWS=$rows timeout -k 10 200 python bench.py --steps 20 --warmup 5
  step $O/b8_rows$rows.log env LJS_ADAM_ROWS=$rows timeout -k 10 200 python bench.py --batch-per-gpu 8 --steps 20 --warmup 5
done
step $O/layer_fp8.log timeout -k 10 200 python bench.py --model layer --fp8 --steps 20 --warmup 5
F4="WORLD_SIZE=4 RANK=0 LOCAL_RANK=0 LJS_DIST_BACKEND=fake MASTER_ADDR=127.0.0.1"
step $O/fake4_2d_fp8.log env $F4 MASTER_PORT=29681 timeout -k 10 300 python bench.py --gpus 4 --mesh 2d --model layer --fp8 --steps 20 --warmup 5
step $O/fake4_dp_fp8.log env $F4 MASTER_PORT=29682 timeout -k 10 300 python bench.py --gpus 4 --mesh dp --model layer --fp8 --steps 20 --warmup 5
step $O/fake4_2d.log env $F4 MASTER_PORT=29683 timeout -k 10 300 python bench.py --gpus 4 --mesh 2d --steps 20 --warmup 5
step $O/fake4_dp.log env $F4 MASTER_PORT=29684 timeout -k 10 300 python bench.py --gpus 4 --mesh dp --steps 20 --warmup 5
cd /tmp
export WORLD_SIZE=4 RANK=0 LOCAL_RANK=0 LJS_DIST_BACKEND=fake MASTER_ADDR=127.0.0.1
step $O/prof_2d_fp8.log env MASTER_PORT=29685 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_2d_fp8 -o run -- python3 $R/bench.py --gpus 4 --mesh 2d --model layer --fp8 --steps 16 --warmup 4
step $O/prof_2d.log env MASTER_PORT=29686 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_2d -o run -- python3 $R/bench.py --gpus 4 --mesh 2d --steps 16 --warmup 4
unset WORLD_SIZE RANK LOCAL_RANK LJS_DIST_BACKEND MASTER_ADDR
step $O/prof_b8.log timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_b8 -o run -- python3 $R/bench.py --batch-per-gpu 8 --steps 16 --warmup 4
step $O/prof_b64.log timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_b64 -o run -- python3 $R/bench.py --steps 16 --warmup 4
echo done
