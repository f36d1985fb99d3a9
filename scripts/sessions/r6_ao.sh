# round-6: head dims other than 64 on the GPU (the torch attention formulation around the HIP
# GEMMs) vs the host run, plus the head_dim-64 block tests
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$PWD/gpurun_out/r6ao
mkdir -p $O
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_e2e.py -k "block_gpu" -p no:cacheprovider > $O/tests.txt 2>&1
echo "rc=$?" >> $O/rc.log
echo done
