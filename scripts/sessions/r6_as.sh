# round-6: the early next-K-tile DMA as the MX layer's default: the fp8 GPU tests, then the
# 1x1 MX-fp8 layer step x3 interleaved with it off (f8_early=0)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=$PWD/gpurun_out/r6as
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
step $O/tests.txt timeout -k 10 600 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_gpu_e2e.py -k "fp8 or mx" -p no:cacheprovider
for rep in 1 2 3; do
  step $O/l8_on_$rep.txt timeout -k 10 300 python scripts/bench_with.py f8_early=1 -- --model layer --fp8 --steps 20 --warmup 5
  step $O/l8_off_$rep.txt timeout -k 10 300 python scripts/bench_with.py f8_early=0 -- --model layer --fp8 --steps 20 --warmup 5
done
for f in $O/l8_*.txt; do echo "$(basename $f) $(grep -o '"ms_per_step": [0-9.]*' $f)"; done > $O/lines.txt
echo done
