cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r3g
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; if [ $rc -ne 0 ]; then echo "rc=$rc: $*" >> $O/rc.log; case $rc in 1|2) ;; *) exit $rc;; esac; fi; }
step $O/tests.log timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_gpu_e2e.py -k "adam or captured or jit or block_gpu or fp8_layer or fp8_ff or fsdp or sum_n or slab"
F4="WORLD_SIZE=4 RANK=0 LOCAL_RANK=0 LJS_DIST_BACKEND=fake MASTER_ADDR=127.0.0.1"
step $O/aten_fake4_2d.log env $F4 MASTER_PORT=29661 LJS_ATEN_TRACE=$O/aten_fake4_2d.txt timeout -k 10 300 python bench.py --gpus 4 --mesh 2d --steps 2 --warmup 2
step $O/aten_b64.log env LJS_ATEN_TRACE=$O/aten_b64.txt timeout -k 10 300 python bench.py --steps 2 --warmup 2
step $O/fsdp4.log env LJS_NUM_DEVICES=4 timeout -k 10 300 python bench.py --model fsdp
step $O/fake4_2d.log env $F4 MASTER_PORT=29664 timeout -k 10 300 python bench.py --gpus 4 --mesh 2d
step $O/fake4_2d_nobatch.log env $F4 MASTER_PORT=29665 LJS_WMAJOR_DW_BATCH=0 timeout -k 10 300 python bench.py --gpus 4 --mesh 2d
for i in 1 2; do
  step $O/b8_e1_$i.log env LJS_EARLY_ADAM=1 timeout -k 10 200 python bench.py --batch-per-gpu 8
  step $O/b8_e0_$i.log env LJS_EARLY_ADAM=0 timeout -k 10 200 python bench.py --batch-per-gpu 8
  step $O/b64_e1_$i.log env LJS_EARLY_ADAM=1 timeout -k 10 200 python bench.py
  step $O/b64_e0_$i.log env LJS_EARLY_ADAM=0 timeout -k 10 200 python bench.py
  step $O/layer8_a1_$i.log env LJS_F8_AUTO=1 timeout -k 10 200 python bench.py --model layer --fp8
  step $O/layer8_a0_$i.log env LJS_F8_AUTO=0 timeout -k 10 200 python bench.py --model layer --fp8
done
step $O/ring.log timeout -k 10 200 python scripts/ring_trace.py
cd /tmp
step $O/prof_b8.log timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_b8 -o run -- python3 $R/bench.py --batch-per-gpu 8 --steps 24 --warmup 6
echo done
