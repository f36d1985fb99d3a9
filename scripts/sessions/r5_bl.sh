# last validation (r5bl) after the Adam ticket removal: full GPU suite, smoke, driver-shape bench lines: full GPU suite, smoke,
# driver-shape bench x3 (B=64) and reference shape x3 (B=8)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r5bl
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
step $O/gpu_tests.txt timeout -k 10 1000 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/
step $O/smoke.txt timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()"
for rep in 1 2 3; do
  step $O/b64_driver_$rep.txt timeout -k 10 300 python bench.py --steps 20 --warmup 5
  step $O/b8_driver_$rep.txt timeout -k 10 300 python bench.py --batch-per-gpu 8 --steps 20 --warmup 5
done
step $O/b64_default.txt timeout -k 10 300 python bench.py
echo done
