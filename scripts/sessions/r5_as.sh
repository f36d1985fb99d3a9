# kernel traces of the MX-fp8 and bf16 transformer layers (current build)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r5as
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
cd /tmp && step $O/prof_fp8.txt timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof_fp8 -o run -- python $R/bench.py --model layer --fp8 --steps 20 --warmup 5
step $O/prof_bf16.txt timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof_bf16 -o run -- python $R/bench.py --model layer --steps 20 --warmup 5
echo done
