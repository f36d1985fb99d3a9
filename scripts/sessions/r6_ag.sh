# round-6: the 2-D layout's overhead over DP on the rehearsal backend (fake-4, rank 0; collectives
# move nothing): kernel traces of the 2-D (2, 2) mesh and of the dp mesh, --secondary off
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r6ag
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
export WORLD_SIZE=4 RANK=0 LOCAL_RANK=0 LJS_DIST_BACKEND=fake MASTER_ADDR=127.0.0.1 MASTER_PORT=29911
step $O/b2d.txt timeout -k 10 300 python bench.py --gpus 4 --mesh 2d --secondary off --steps 20 --warmup 5
step $O/bdp.txt timeout -k 10 300 python bench.py --gpus 4 --secondary off --steps 20 --warmup 5
cd /tmp
step $O/prof_2d.log timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof_2d -o run -- python3 $R/bench.py --gpus 4 --mesh 2d --secondary off --steps 20 --warmup 5
step $O/prof_dp.log timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof_dp -o run -- python3 $R/bench.py --gpus 4 --secondary off --steps 20 --warmup 5
cd $R
python scripts/kstats.py $O/prof_2d/run_results.db --steps 86 > $O/k2d.md 2>&1
python scripts/kstats.py $O/prof_dp/run_results.db --steps 86 > $O/kdp.md 2>&1
echo done
