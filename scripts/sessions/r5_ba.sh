# held weight-gradient jobs per device (locked, run on their own stream) + thread-local group
# recording: the grouped / deferred / e2e / multi-device tests, then B=64 and B=8 once each
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r5ba
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
step $O/tests.txt timeout -k 10 700 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/ -k "gemm_group or grouped or deferred or e2e or multi_gpu or capture or weight_gather or fsdp or proxy"
step $O/b64.txt timeout -k 10 300 python bench.py
step $O/b8.txt timeout -k 10 300 python bench.py --batch-per-gpu 8
echo done
