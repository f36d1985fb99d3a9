set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r3d
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "attn or attention or mse or sum_n or transpose" > $O/tests.log 2>&1
timeout -k 10 120 python scripts/attn_layout.py > $O/layout.log 2>&1
cd /tmp
for v in 0 1; do
  LJS_ATTN_FWD_PROG=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/kt_prog$v -o run -- python3 $R/scripts/attn_one.py fwd 64 256 8 20 > $O/kt_prog$v.log 2>&1
  LJS_ATTN_FWD_PROG=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/kt8_prog$v -o run -- python3 $R/scripts/attn_one.py fwd 8 256 8 20 > $O/kt8_prog$v.log 2>&1
done
cd $R
for i in 1 2; do
  for v in 0 1; do LJS_ATTN_FWD_PROG=$v timeout -k 10 200 python bench.py >> $O/b64_prog$v.log 2>&1; done
done
timeout -k 10 200 python bench.py --loss mse > $O/b64_mse.log 2>&1
timeout -k 10 200 python bench.py --batch-per-gpu 8 > $O/b8.log 2>&1
WORLD_SIZE=4 RANK=0 LOCAL_RANK=0 LJS_DIST_BACKEND=fake MASTER_ADDR=127.0.0.1 MASTER_PORT=29651 timeout -k 10 300 python bench.py --gpus 4 --mesh 2d > $O/fake4_2d.log 2>&1
WORLD_SIZE=4 RANK=0 LOCAL_RANK=0 LJS_DIST_BACKEND=fake MASTER_ADDR=127.0.0.1 MASTER_PORT=29652 timeout -k 10 300 python bench.py --gpus 4 --mesh dp > $O/fake4_dp.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_mse -o run -- python bench.py --loss mse --steps 24 --warmup 6 > $O/prof_mse.log 2>&1
timeout -k 10 180 python scripts/fp8_tiles.py 20 > $O/fp8_tiles.log 2>&1
echo done
