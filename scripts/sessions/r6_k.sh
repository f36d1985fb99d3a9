# round-6: fused attention phase with shared K/V fragments for both query sub-tiles (fwd_tile2) A/B
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r6k
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
V=$R/learning_jax_sharding_amd/_lib/variants
step $O/tests_k.txt timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "qkv_attn"
step $O/tests_e.txt timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_e2e.py -k "fused_qkv"
for rep in 1 2 3; do
  step $O/b64_t2_$rep.txt timeout -k 10 300 python bench.py --steps 20 --warmup 5
  step $O/b64_t1_$rep.txt timeout -k 10 300 env LJS_KERNELS_LIB=$V/tile1/libljs_kernels.so python bench.py --steps 20 --warmup 5
done
for f in $O/b*_*.txt; do echo "$(basename $f) $(grep -o '"ms_per_step": [0-9.]*' $f)"; done > $O/lines.txt
cd /tmp
step $O/prof_b64.log timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof_b64 -o run -- python3 $R/bench.py --steps 20 --warmup 5
cd $R
python scripts/kstats.py $O/prof_b64/run_results.db --steps 86 > $O/b64_kernels.md 2>&1
echo done
