cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r3ad
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; if [ $rc -ne 0 ]; then echo "rc=$rc: $*" >> $O/rc.log; case $rc in 1|2) ;; *) exit $rc;; esac; fi; }
for i in 1 2; do
  for e in 0 2 1; do
    step $O/b64_e${e}_$i.log env LJS_EARLY_ADAM=$e timeout -k 10 200 python bench.py
    step $O/b8_e${e}_$i.log env LJS_EARLY_ADAM=$e timeout -k 10 200 python bench.py --batch-per-gpu 8
  done
done
cd /tmp
step $O/prof_b64_e2.log env LJS_EARLY_ADAM=2 timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof_b64_e2 -o run -- python3 $R/bench.py --steps 16 --warmup 4
echo done
