cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r3f
mkdir -p $O
# step LOG cmd...: a failing check (rc 1/2) does not stop the session; a fault, abort or time limit does
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; if [ $rc -ne 0 ]; then echo "rc=$rc: $*" >> $O/rc.log; case $rc in 1|2) ;; *) exit $rc;; esac; fi; }
F4="WORLD_SIZE=4 RANK=0 LOCAL_RANK=0 LJS_DIST_BACKEND=fake MASTER_ADDR=127.0.0.1"
step $O/tests_k.log timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "fp8 or sum_n or transpose"
step $O/tests_e2e.log timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_e2e.py -k "fsdp or block_gpu"
step $O/fp8_tiles.log timeout -k 10 300 python scripts/fp8_tiles.py 20
step $O/aten_fake4_2d.log env $F4 MASTER_PORT=29661 LJS_ATEN_TRACE=$O/aten_fake4_2d.txt timeout -k 10 300 python bench.py --gpus 4 --mesh 2d --steps 2 --warmup 2
step $O/aten_fsdp4.log env LJS_NUM_DEVICES=4 LJS_ATEN_TRACE=$O/aten_fsdp4.txt timeout -k 10 300 python bench.py --model fsdp --steps 2 --warmup 2
step $O/fsdp4.log env LJS_NUM_DEVICES=4 timeout -k 10 300 python bench.py --model fsdp
step $O/case5_4.log env LJS_NUM_DEVICES=4 timeout -k 10 300 python bench.py --mesh 4x1 --rules case5
step $O/fake4_2d.log env $F4 MASTER_PORT=29663 timeout -k 10 300 python bench.py --gpus 4 --mesh 2d
cd /tmp
step $O/prof_fsdp4.log env LJS_NUM_DEVICES=4 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_fsdp4 -o run -- python3 $R/bench.py --model fsdp --steps 24 --warmup 6
step $O/prof_fake4_2d.log env $F4 MASTER_PORT=29662 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_fake4_2d -o run -- python3 $R/bench.py --gpus 4 --mesh 2d --steps 24 --warmup 6
echo done
