cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r3m
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; if [ $rc -ne 0 ]; then echo "rc=$rc: $*" >> $O/rc.log; case $rc in 1|2) ;; *) exit $rc;; esac; fi; }
F4="WORLD_SIZE=4 RANK=0 LOCAL_RANK=0 LJS_DIST_BACKEND=fake MASTER_ADDR=127.0.0.1"
step $O/tests.log timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "large_tiles or fp8_transformer or transpose or swap"
for i in 1 2; do
  step $O/layer8_cs1_$i.log env LJS_F8_FUSED_COLSUM=1 timeout -k 10 200 python bench.py --model layer --fp8
  step $O/layer8_cs0_$i.log env LJS_F8_FUSED_COLSUM=0 timeout -k 10 200 python bench.py --model layer --fp8
done
for t in 128160 128320; do
  step $O/layer8_$t.log env LJS_F8_N640_TILE=$t timeout -k 10 200 python bench.py --model layer --fp8
done
step $O/fake4_2d.log env $F4 MASTER_PORT=29671 timeout -k 10 300 python bench.py --gpus 4 --mesh 2d
step $O/fake4_dp.log env $F4 MASTER_PORT=29672 timeout -k 10 300 python bench.py --gpus 4 --mesh dp
echo done
