cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r3ab
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; if [ $rc -ne 0 ]; then echo "rc=$rc: $*" >> $O/rc.log; case $rc in 1|2) ;; *) exit $rc;; esac; fi; }
for i in 1 2; do
  step $O/base_$i.log timeout -k 10 200 python bench.py
  step $O/t12884_r1_$i.log env LJS_DW_BIG_TILE=12884 timeout -k 10 200 python bench.py
  step $O/t12884_r2_$i.log env LJS_DW_BIG_TILE=12884 LJS_DW_BIG_ROUNDS=2 timeout -k 10 200 python bench.py
  step $O/t12884_r3_$i.log env LJS_DW_BIG_TILE=12884 LJS_DW_BIG_ROUNDS=3 timeout -k 10 200 python bench.py
done
cd /tmp
for c in "base" "t12884_r2:LJS_DW_BIG_TILE=12884 LJS_DW_BIG_ROUNDS=2"; do
  tag=${c%%:*}; ev=${c#*:}; [ "$tag" = "$c" ] && ev=""
  step $O/prof_$tag.log env $ev timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$tag -o run -- python3 $R/bench.py --steps 16 --warmup 4
done
echo done
