# DMA-issue vs MFMA interference probe (scripts/probe_dma_mfma.hip)
cd "$GRAFT_REPO_ROOT"
O=$PWD/gpurun_out/r5d
mkdir -p $O
timeout -k 10 120 ./scripts/probe_dma_mfma.bin > $O/probe.log 2>&1
echo rc=$?
