# round-6: aten + HIP-glue call sites of the fake-4 2-D step (which pack / transpose launches run,
# and from where)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$PWD/gpurun_out/r6ah
mkdir -p $O
export WORLD_SIZE=4 RANK=0 LOCAL_RANK=0 LJS_DIST_BACKEND=fake MASTER_ADDR=127.0.0.1 MASTER_PORT=29913
LJS_ATEN_TRACE=$O/glue_2d.txt timeout -k 10 300 python bench.py --gpus 4 --mesh 2d --secondary off --steps 5 --warmup 2 > $O/b2d.txt 2>&1
echo "rc=$?" >> $O/rc.log
echo done
