set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r3a
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_e2e.py tests/test_rehearsal_gpu.py > $O/tests.log 2>&1
timeout -k 10 200 python bench.py > $O/b64.log 2>&1
timeout -k 10 200 python bench.py --loss mse > $O/b64_mse.log 2>&1
timeout -k 10 200 python bench.py --batch-per-gpu 8 > $O/b8.log 2>&1
timeout -k 10 200 python bench.py --gpus 1 --batch-per-gpu 64 --steps 20 > $O/b64_g1.log 2>&1
LJS_NUM_DEVICES=4 timeout -k 10 300 python bench.py --mesh 2x2 > $O/v2x2.log 2>&1
LJS_NUM_DEVICES=4 timeout -k 10 300 python bench.py --mesh 4x1 > $O/v4x1.log 2>&1
WORLD_SIZE=4 RANK=0 LOCAL_RANK=0 LJS_DIST_BACKEND=fake MASTER_ADDR=127.0.0.1 MASTER_PORT=29650 timeout -k 10 300 python bench.py --gpus 4 --mesh 2d > $O/fake4_2d.log 2>&1
WORLD_SIZE=4 RANK=0 LOCAL_RANK=0 LJS_DIST_BACKEND=fake MASTER_ADDR=127.0.0.1 MASTER_PORT=29651 timeout -k 10 300 python bench.py --gpus 4 --mesh dp > $O/fake4_dp.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_mse -o run -- python bench.py --loss mse --steps 24 --warmup 6 > $O/prof_mse.log 2>&1
LJS_NUM_DEVICES=4 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_v2x2 -o run -- python bench.py --mesh 2x2 --steps 24 --warmup 6 > $O/prof_v2x2.log 2>&1
WORLD_SIZE=4 RANK=0 LOCAL_RANK=0 LJS_DIST_BACKEND=fake MASTER_ADDR=127.0.0.1 MASTER_PORT=29652 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_fake4_2d -o run -- python bench.py --gpus 4 --mesh 2d --steps 24 --warmup 6 > $O/prof_fake4_2d.log 2>&1
echo done
