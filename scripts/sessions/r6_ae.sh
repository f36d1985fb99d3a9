# round-6: stream-safe segmented-capture cuts (a cut on a forked stream joins it first) and no
# side-stream forks where collectives cut the capture (graphs.forks_ok): the GPU tests of the
# capture paths, then the 2-D gloo bench that failed in r6ad and the N=2 gloo bench with its
# 2-D secondary (r6ab)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$PWD/gpurun_out/r6ae
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
step $O/tests.txt timeout -k 10 700 python -u -m pytest -v --timeout 600 --timeout-method thread \
  tests/test_multi_gpu_capture_gpu.py tests/test_distributed_gpu.py -p no:cacheprovider
export LJS_DIST_BACKEND=gloo
step $O/gloo2_2d.txt timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29711 bench.py --gpus 2 --mesh 2d --secondary off --steps 10 --warmup 3
step $O/gloo2.txt timeout -k 10 420 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29721 bench.py --gpus 2 --steps 10 --warmup 3
echo done
