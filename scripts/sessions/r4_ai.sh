# steps per captured graph at --steps 20, the small side: G = 2, 4, 5
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r4ai
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then case $rc in 1|2) ;; *) exit $rc;; esac; fi; }
for i in 1 2 3; do
for g in 2 4 5; do
step $O/drv_g${g}_$i.log timeout -k 10 200 python bench.py --steps 20 --warmup 5 --graph-steps $g
step $O/b8_g${g}_$i.log timeout -k 10 200 python bench.py --batch-per-gpu 8 --steps 20 --warmup 5 --graph-steps $g
done
done
for f in $O/drv*.log $O/b8*.log; do grep -h ms_per_step $f | python -c "
import sys,json
for l in sys.stdin:
    r=json.loads(l); print('$(basename $f)', r['ms_per_step'], r['value'], r.get('warmup'))
" >> $O/summary.txt || true; done
echo done
