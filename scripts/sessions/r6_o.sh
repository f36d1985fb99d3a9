# round-6 validation of the current build: every GPU test, smoke(), the driver-shape bench and
# the reference shape, a fresh B=64 trace
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r6o
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
step $O/tests.txt timeout -k 10 1500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/
step $O/smoke.txt timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()"
step $O/b64_1.txt timeout -k 10 300 python bench.py --steps 20 --warmup 5
step $O/b64_2.txt timeout -k 10 300 python bench.py --steps 20 --warmup 5
step $O/b8_1.txt timeout -k 10 300 python bench.py --batch-per-gpu 8 --steps 20 --warmup 5
step $O/def_1.txt timeout -k 10 300 python bench.py
step $O/l8_1.txt timeout -k 10 300 python bench.py --model layer --fp8 --steps 20 --warmup 5
for f in $O/b*_*.txt $O/def_*.txt $O/l8_*.txt; do echo "$(basename $f) $(grep -o '"ms_per_step": [0-9.]*' $f)"; done > $O/lines.txt
echo done
