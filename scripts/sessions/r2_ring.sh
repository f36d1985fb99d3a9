set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_e2e.py -x -q --timeout 200 --timeout-method thread -k "ring" > gpurun_out/r2r_tests.log 2>&1
timeout -k 10 120 python scripts/ring_trace.py > gpurun_out/r2r_time.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/r2r_prof -o prof -- python scripts/ring_trace.py > gpurun_out/r2r_prof.log 2>&1
