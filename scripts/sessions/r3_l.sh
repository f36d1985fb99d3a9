cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r3l
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; if [ $rc -ne 0 ]; then echo "rc=$rc: $*" >> $O/rc.log; case $rc in 1|2) ;; *) exit $rc;; esac; fi; }
step $O/gpu_tests.log timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/
step $O/smoke.log timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
for t in 256160 128160 128320; do
  step $O/layer8_$t.log env LJS_F8_N640_TILE=$t timeout -k 10 200 python bench.py --model layer --fp8
done
for i in 1 2; do
  step $O/layer8_cs1_$i.log env LJS_F8_FUSED_COLSUM=1 timeout -k 10 200 python bench.py --model layer --fp8
  step $O/layer8_cs0_$i.log env LJS_F8_FUSED_COLSUM=0 timeout -k 10 200 python bench.py --model layer --fp8
done
step $O/b64.log timeout -k 10 200 python bench.py
echo done
