cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r3j
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; if [ $rc -ne 0 ]; then echo "rc=$rc: $*" >> $O/rc.log; case $rc in 1|2) ;; *) exit $rc;; esac; fi; }
F4="WORLD_SIZE=4 RANK=0 LOCAL_RANK=0 LJS_DIST_BACKEND=fake MASTER_ADDR=127.0.0.1"
step $O/tests.log timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_e2e.py tests/test_distributed_gpu.py tests/test_kernels_gpu.py -k "block_gpu or fsdp or dp_check or distributed or fp8 or quant or mx"
step $O/probe.log timeout -k 10 120 python scripts/cvt_scalef_probe.py
step $O/fake4_2d.log env $F4 MASTER_PORT=29671 timeout -k 10 300 python bench.py --gpus 4 --mesh 2d
step $O/fake4_dp.log env $F4 MASTER_PORT=29672 timeout -k 10 300 python bench.py --gpus 4 --mesh dp
step $O/v2x2.log env LJS_NUM_DEVICES=4 timeout -k 10 300 python bench.py --mesh 2x2
step $O/fsdp4.log env LJS_NUM_DEVICES=4 timeout -k 10 300 python bench.py --model fsdp
step $O/case5_4.log env LJS_NUM_DEVICES=4 timeout -k 10 300 python bench.py --mesh 4x1 --rules case5
step $O/layer8.log timeout -k 10 200 python bench.py --model layer --fp8
step $O/layer.log timeout -k 10 200 python bench.py --model layer
step $O/fp8_tiles.log timeout -k 10 300 python scripts/fp8_tiles.py 20 1282,256160,3128256
for r in 16 32 64; do step $O/b8_rows$r.log env LJS_ADAM_ROWS=$r timeout -k 10 200 python bench.py --batch-per-gpu 8; done
step $O/b64.log timeout -k 10 200 python bench.py
cd /tmp
step $O/prof_v2x2.log env LJS_NUM_DEVICES=4 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_v2x2 -o run -- python3 $R/bench.py --mesh 2x2 --steps 24 --warmup 6
step $O/prof_case5.log env LJS_NUM_DEVICES=4 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_case5 -o run -- python3 $R/bench.py --mesh 4x1 --rules case5 --steps 24 --warmup 6
echo done
