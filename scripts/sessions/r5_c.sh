# per-CU LDS-DMA fill rate vs bytes in flight (scripts/probe_fill.hip) and the older load probe
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r5c
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then case $rc in 1|2) ;; *) exit $rc;; esac; fi; }
step $O/fill.log timeout -k 10 120 ./scripts/probe_fill.bin
step $O/load.log timeout -k 10 120 ./scripts/probe_load_bw.bin
echo done
