# round-6: the peer-memory (IPC) collectives in the driver's launch form: 2 ranks sharing the one
# GPU over gloo with LJS_P2P=1 (peer groups built on one device), the 2-D (1, 2) mesh: collectives
# <= 1 MiB through the captured IPC kernels, the rest through gloo (capture cuts)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$PWD/gpurun_out/r6am
mkdir -p $O
export LJS_DIST_BACKEND=gloo LJS_P2P=1
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29731 bench.py --gpus 2 --mesh 1x2 --secondary off --steps 10 --warmup 3 > $O/p2p_1x2.txt 2>&1
echo "rc=$?" >> $O/rc.log
echo done
