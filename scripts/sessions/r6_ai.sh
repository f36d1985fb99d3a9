# round-6: which weight's transposed bf16 shadow the fake-4 2-D step re-casts every step
# (cast_transpose_f32_bf16, 1 call / step in profiles/r6ag_fake4_2d_kernels.md)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$PWD/gpurun_out/r6ai
mkdir -p $O
export WORLD_SIZE=4 RANK=0 LOCAL_RANK=0 LJS_DIST_BACKEND=fake MASTER_ADDR=127.0.0.1 MASTER_PORT=29915
LJS_SHADOW_TRACE=1 timeout -k 10 300 python bench.py --gpus 4 --mesh 2d --secondary off --steps 5 --warmup 2 --min-warmup 2 --no-graph > $O/b2d.txt 2>&1
echo "rc=$?" >> $O/rc.log
echo done
