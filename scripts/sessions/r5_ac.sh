# B=64 A/B x3 interleaved: default vs the 256x128 tile for the [T][512] dX GEMM
# (LJS_GEMM_2561_MIN_N=512) vs the persistent double-buffered attention forward (LJS_ATTN_FWD_RES=108)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r5ac
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
step $O/tests.txt timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu -k "attention_fwd or attn_fwd or fwd_res or pers" tests/test_kernels_gpu.py
for rep in 1 2 3; do
  step $O/default_$rep.txt timeout -k 10 300 python bench.py
  LJS_GEMM_2561_MIN_N=512 step $O/dh2561_$rep.txt timeout -k 10 300 python bench.py
  LJS_ATTN_FWD_RES=108 step $O/fwdpers_$rep.txt timeout -k 10 300 python bench.py
done
echo done
