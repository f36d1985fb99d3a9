cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r3al
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; if [ $rc -ne 0 ]; then echo "rc=$rc: $*" >> $O/rc.log; case $rc in 1|2) ;; *) exit $rc;; esac; fi; }
for i in 1 2; do
  step $O/s20w5_$i.log timeout -k 10 200 python bench.py --steps 20 --warmup 5
  step $O/s40w5_$i.log timeout -k 10 200 python bench.py --steps 40 --warmup 5
  step $O/s20w40_$i.log timeout -k 10 200 python bench.py --steps 20 --warmup 40
  step $O/s16w5_$i.log timeout -k 10 200 python bench.py --steps 16 --warmup 5
  step $O/s96w10_$i.log timeout -k 10 200 python bench.py --steps 96 --warmup 10
done
echo done
