# full GPU suite, then register-staged cast-on-load + bf16 slabs A/B, 2-D glue trace / table
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r4j
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then case $rc in 1|2) ;; *) exit $rc;; esac; fi; }
step $O/gpu_tests.log timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/
if grep -q " failed\|[0-9] error" $O/gpu_tests.log; then echo "tests failed"; tail -40 $O/gpu_tests.log; exit 1; fi
step $O/qkv32.log timeout -k 10 200 python scripts/gemm_pp_bench.py qkv32 qkv
for i in 1 2; do
step $O/drv_def_$i.log timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5
step $O/drv_col0_$i.log env LJS_CAST_ON_LOAD=0 timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5
step $O/drv_s16_$i.log env LJS_SLAB_BF16=1 timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5
step $O/drv_both_$i.log env LJS_SLAB_BF16=1 LJS_CAST_ON_LOAD=0 timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5
done
step $O/b8_def.log timeout -k 10 200 python bench.py --batch-per-gpu 8 --steps 20 --warmup 5
step $O/b8_col0.log env LJS_CAST_ON_LOAD=0 timeout -k 10 200 python bench.py --batch-per-gpu 8 --steps 20 --warmup 5
step $O/b8_s16.log env LJS_SLAB_BF16=1 timeout -k 10 200 python bench.py --batch-per-gpu 8 --steps 20 --warmup 5
F4="WORLD_SIZE=4 RANK=0 LOCAL_RANK=0 LJS_DIST_BACKEND=fake MASTER_ADDR=127.0.0.1"
step $O/trace_2d.log env $F4 MASTER_PORT=29721 LJS_ATEN_TRACE=$O/aten_2d.txt timeout -k 10 300 python -X faulthandler bench.py --gpus 4 --mesh 2d --steps 2 --warmup 2 --min-warmup 0
step $O/fake4_2d.log env $F4 MASTER_PORT=29722 timeout -k 10 300 python bench.py --gpus 4 --mesh 2d --steps 20 --warmup 5
step $O/fake4_2d_split.log env $F4 MASTER_PORT=29723 LJS_ATTN_BWD_FUSED=0 timeout -k 10 300 python bench.py --gpus 4 --mesh 2d --steps 20 --warmup 5
step $O/fake4_dp.log env $F4 MASTER_PORT=29724 timeout -k 10 300 python bench.py --gpus 4 --mesh dp --steps 20 --warmup 5
cd /tmp
step $O/prof_b64.log timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_b64 -o run -- python3 $R/bench.py --steps 16 --warmup 4
step $O/prof_b8.log timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_b8 -o run -- python3 $R/bench.py --batch-per-gpu 8 --steps 16 --warmup 4
export WORLD_SIZE=4 RANK=0 LOCAL_RANK=0 LJS_DIST_BACKEND=fake MASTER_ADDR=127.0.0.1
step $O/prof_2d.log env MASTER_PORT=29725 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_2d -o run -- python3 $R/bench.py --gpus 4 --mesh 2d --steps 16 --warmup 4
echo done
