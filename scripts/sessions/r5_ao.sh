# the pair pick now declines pairs whose separate launches estimate lower (the FF block's): layer
# bf16 / fp8 and the attention step, grouping on vs off
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r5ao
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
step $O/tests.txt timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_epilogue_gpu.py tests/test_gpu_e2e.py
for rep in 1 2; do
  step $O/layer_group_$rep.txt timeout -k 10 300 python bench.py --model layer
  LJS_DW_GROUP=0 step $O/layer_sep_$rep.txt timeout -k 10 300 python bench.py --model layer
  step $O/fp8_group_$rep.txt timeout -k 10 300 python bench.py --model layer --fp8
  step $O/b64_group_$rep.txt timeout -k 10 300 python bench.py
done
echo done
