set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r3c
mkdir -p $O
WORLD_SIZE=4 RANK=0 LOCAL_RANK=0 LJS_DIST_BACKEND=fake MASTER_ADDR=127.0.0.1 MASTER_PORT=29650 LJS_SHADOW_TRACE=1 timeout -k 10 200 python bench.py --gpus 4 --mesh 2d --steps 3 --warmup 3 --no-graph --batch-per-gpu 8 > $O/fake2d_trace.log 2>&1
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_e2e.py tests/test_kernels_gpu.py -k "fwd_inkernel or ring or mse or block_gpu or captured or detached" > $O/tests.log 2>&1
timeout -k 10 200 python bench.py > $O/b64.log 2>&1
timeout -k 10 200 python bench.py --loss mse > $O/b64_mse.log 2>&1
WORLD_SIZE=4 RANK=0 LOCAL_RANK=0 LJS_DIST_BACKEND=fake MASTER_ADDR=127.0.0.1 MASTER_PORT=29651 timeout -k 10 300 python bench.py --gpus 4 --mesh 2d > $O/fake4_2d.log 2>&1
WORLD_SIZE=4 RANK=0 LOCAL_RANK=0 LJS_DIST_BACKEND=fake MASTER_ADDR=127.0.0.1 MASTER_PORT=29652 timeout -k 10 300 python bench.py --gpus 4 --mesh dp > $O/fake4_dp.log 2>&1
LJS_NUM_DEVICES=4 timeout -k 10 300 python bench.py --mesh 2x2 > $O/v2x2.log 2>&1
LJS_NUM_DEVICES=4 timeout -k 10 300 python bench.py --model fsdp > $O/fsdp4.log 2>&1
LJS_NUM_DEVICES=4 timeout -k 10 300 python bench.py --mesh 4x1 --rules case5 > $O/case5_4.log 2>&1
LJS_NUM_DEVICES=4 timeout -k 10 300 python bench.py --mesh 1x4 --seq 1024 --batch-per-gpu 4 > $O/sp4_ag.log 2>&1
WORLD_SIZE=4 RANK=0 LOCAL_RANK=0 LJS_DIST_BACKEND=fake MASTER_ADDR=127.0.0.1 MASTER_PORT=29653 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_fake4_2d -o run -- python bench.py --gpus 4 --mesh 2d --steps 24 --warmup 6 > $O/prof_fake4_2d.log 2>&1
LJS_NUM_DEVICES=4 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_fsdp4 -o run -- python bench.py --model fsdp --steps 24 --warmup 6 > $O/prof_fsdp4.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_mse -o run -- python bench.py --loss mse --steps 24 --warmup 6 > $O/prof_mse.log 2>&1
echo done
