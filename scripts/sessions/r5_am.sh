# full GPU suite without -x: list every test the grouped weight-gradient pair changes
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$PWD/gpurun_out/r5am
mkdir -p $O
timeout -k 10 1000 python -u -m pytest -q -rf --timeout 120 --timeout-method thread -m gpu tests/ > $O/gpu_tests.txt 2>&1; echo "rc=$?" >> $O/gpu_tests.txt
