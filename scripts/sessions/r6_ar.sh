# round-6: MX-fp8 up projection / dA with the next K-tile's DMA issued ahead of the fragment
# reads (tile 1289): bit-exact tests, then the up-projection probe (all tiles)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$PWD/gpurun_out/r6ar
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
step $O/tests.txt timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "early_dma or 8wave_tiles_match" -p no:cacheprovider
step $O/probe.txt timeout -k 10 300 python scripts/fp8_upproj_probe.py 20
step $O/probe2.txt timeout -k 10 300 python scripts/fp8_upproj_probe.py 20
echo done
