set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r3b
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_e2e.py tests/test_distributed_gpu.py tests/test_rehearsal_gpu.py > $O/tests.log 2>&1
timeout -k 10 200 python bench.py > $O/b64.log 2>&1
WORLD_SIZE=4 RANK=0 LOCAL_RANK=0 LJS_DIST_BACKEND=fake MASTER_ADDR=127.0.0.1 MASTER_PORT=29650 timeout -k 10 300 python bench.py --gpus 4 --mesh 2d > $O/fake4_2d.log 2>&1
WORLD_SIZE=4 RANK=0 LOCAL_RANK=0 LJS_DIST_BACKEND=fake MASTER_ADDR=127.0.0.1 MASTER_PORT=29651 timeout -k 10 300 python bench.py --gpus 4 --mesh dp > $O/fake4_dp.log 2>&1
LJS_NUM_DEVICES=4 timeout -k 10 300 python bench.py --mesh 2x2 > $O/v2x2.log 2>&1
LJS_NUM_DEVICES=4 timeout -k 10 300 python bench.py --model fsdp > $O/fsdp4.log 2>&1
LJS_NUM_DEVICES=4 timeout -k 10 300 python bench.py --mesh 4x1 --rules case5 > $O/case5_4.log 2>&1
WORLD_SIZE=4 RANK=0 LOCAL_RANK=0 LJS_DIST_BACKEND=fake MASTER_ADDR=127.0.0.1 MASTER_PORT=29652 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_fake4_2d -o run -- python bench.py --gpus 4 --mesh 2d --steps 24 --warmup 6 > $O/prof_fake4_2d.log 2>&1
LJS_NUM_DEVICES=4 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_fsdp4 -o run -- python bench.py --model fsdp --steps 24 --warmup 6 > $O/prof_fsdp4.log 2>&1
echo done
