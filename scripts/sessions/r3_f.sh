set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r3f
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "fp8 or sum_n or transpose" > $O/tests_k.log 2>&1
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_e2e.py -k "fsdp or block_gpu" > $O/tests_e2e.log 2>&1
timeout -k 10 300 python scripts/fp8_tiles.py 20 > $O/fp8_tiles.log 2>&1
F4="WORLD_SIZE=4 RANK=0 LOCAL_RANK=0 LJS_DIST_BACKEND=fake MASTER_ADDR=127.0.0.1"
env $F4 MASTER_PORT=29661 LJS_ATEN_TRACE=$O/aten_fake4_2d.txt timeout -k 10 300 python bench.py --gpus 4 --mesh 2d --steps 2 --warmup 2 > $O/aten_fake4_2d.log 2>&1
LJS_NUM_DEVICES=4 LJS_ATEN_TRACE=$O/aten_fsdp4.txt timeout -k 10 300 python bench.py --model fsdp --steps 2 --warmup 2 > $O/aten_fsdp4.log 2>&1
LJS_NUM_DEVICES=4 timeout -k 10 300 python bench.py --model fsdp > $O/fsdp4.log 2>&1
LJS_NUM_DEVICES=4 timeout -k 10 300 python bench.py --mesh 4x1 --rules case5 > $O/case5_4.log 2>&1
cd /tmp
LJS_NUM_DEVICES=4 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_fsdp4 -o run -- python3 $R/bench.py --model fsdp --steps 24 --warmup 6 > $O/prof_fsdp4.log 2>&1
env $F4 MASTER_PORT=29662 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_fake4_2d -o run -- python3 $R/bench.py --gpus 4 --mesh 2d --steps 24 --warmup 6 > $O/prof_fake4_2d.log 2>&1
echo done
