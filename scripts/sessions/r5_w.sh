# 2-D glue inventory on the current build: aten + HIP-glue trace of one fake-4 2-D step (bf16
# block) and of the 2-D MX-fp8 layer step
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r5w
mkdir -p $O
F4="WORLD_SIZE=4 RANK=0 LOCAL_RANK=0 LJS_DIST_BACKEND=fake MASTER_ADDR=127.0.0.1"
env $F4 MASTER_PORT=29941 LJS_ATEN_TRACE=$O/glue_2d.txt timeout -k 10 300 python bench.py --gpus 4 --mesh 2d --steps 4 --warmup 2 --min-warmup 0 > $O/glue_2d.log 2>&1 || exit 3
env $F4 MASTER_PORT=29942 LJS_ATEN_TRACE=$O/glue_2d_fp8.txt timeout -k 10 300 python bench.py --gpus 4 --mesh 2d --model layer --fp8 --steps 4 --warmup 2 --min-warmup 0 > $O/glue_2d_fp8.log 2>&1 || exit 3
echo done
