# round-6: the secondary configurations on the fused-attention build (one run each)
# secondary configurations on the final round-5 build (one run each; r4aa was the last full set)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r6u
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
step $O/s4096.log timeout -k 10 300 python bench.py --seq 4096 --batch-per-gpu 4
step $O/s1024.log timeout -k 10 300 python bench.py --seq 1024 --batch-per-gpu 16
step $O/ff.log timeout -k 10 300 python bench.py --model ff
step $O/ff8.log timeout -k 10 300 python bench.py --model ff --fp8
step $O/fsdp4096.log timeout -k 10 300 python bench.py --model fsdp --dim 4096
step $O/fsdp4v.log env LJS_NUM_DEVICES=4 timeout -k 10 300 python bench.py --model fsdp
step $O/case5v.log env LJS_NUM_DEVICES=4 timeout -k 10 300 python bench.py --mesh 4x1 --rules case5
step $O/v2x2.log env LJS_NUM_DEVICES=4 timeout -k 10 300 python bench.py --mesh 2x2
step $O/mse.log timeout -k 10 300 python bench.py --loss mse
step $O/fwd.log timeout -k 10 300 python bench.py --mode fwd
step $O/layer.log timeout -k 10 300 python bench.py --model layer
for f in $O/*.log; do echo "$(basename $f) $(grep -o "\"ms_per_step\": [0-9.]*" $f | head -1)"; done > $O/lines.txt
echo done
