cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r3af
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; if [ $rc -ne 0 ]; then echo "rc=$rc: $*" >> $O/rc.log; case $rc in 1|2) ;; *) exit $rc;; esac; fi; }
for i in 1 2 3; do
  step $O/base_$i.log timeout -k 10 200 python bench.py
  step $O/prio_$i.log env LJS_ATTN_PRIO=1 timeout -k 10 200 python bench.py
  step $O/prog_$i.log env LJS_ATTN_FWD_PROG=1 timeout -k 10 200 python bench.py
done
cd /tmp
for c in base prio prog; do
  ev=""; [ $c = prio ] && ev="LJS_ATTN_PRIO=1"; [ $c = prog ] && ev="LJS_ATTN_FWD_PROG=1"
  step $O/pa_$c.log env $ev LJS_X=1 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/pa_$c -o run -- python3 $R/scripts/attn_one.py bwd 64 256 8 30
done
echo done
