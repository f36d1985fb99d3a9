# the weight-gradient pair on the transformer layer (bf16 and MX-fp8 FF): LJS_DW_GROUP=1 vs 0, x2
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r5an
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
for rep in 1 2; do
  step $O/layer_group_$rep.txt timeout -k 10 300 python bench.py --model layer
  LJS_DW_GROUP=0 step $O/layer_sep_$rep.txt timeout -k 10 300 python bench.py --model layer
  step $O/fp8_group_$rep.txt timeout -k 10 300 python bench.py --model layer --fp8
  LJS_DW_GROUP=0 step $O/fp8_sep_$rep.txt timeout -k 10 300 python bench.py --model layer --fp8
done
cd /tmp && step $O/prof_layer.txt timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_layer -o run -- python $R/bench.py --model layer --steps 20 --warmup 5
echo done
