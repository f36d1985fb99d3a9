# round-6: the 32x32x16-MFMA lean GEMM (correctness + isolated A/B at the step shapes) and the
# sched_group_barrier variant; step-level A/B of both as variant libraries, x3 interleaved
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r6e
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
step $O/tests.txt timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "lean32 or lean_bit_exact or fp8_quantization or fp8_ff_block"
step $O/mf32_ab.txt timeout -k 10 300 python scripts/gemm_mf32_ab.py
V=$R/learning_jax_sharding_amd/_lib/variants
for rep in 1 2 3; do
  step $O/b64_base_$rep.txt timeout -k 10 300 python bench.py --steps 20 --warmup 5
  step $O/b64_mf32_$rep.txt timeout -k 10 300 env LJS_KERNELS_LIB=$V/mf32/libljs_kernels.so python bench.py --steps 20 --warmup 5
  step $O/b64_sgb_$rep.txt timeout -k 10 300 env LJS_KERNELS_LIB=$V/sgb/libljs_kernels.so python bench.py --steps 20 --warmup 5
  step $O/b64_fastidx_$rep.txt timeout -k 10 300 env LJS_KERNELS_LIB=$V/fastidx/libljs_kernels.so python bench.py --steps 20 --warmup 5
done
for rep in 1 2; do
  step $O/b8_base_$rep.txt timeout -k 10 300 python bench.py --batch-per-gpu 8 --steps 20 --warmup 5
  step $O/b8_mf32_$rep.txt timeout -k 10 300 env LJS_KERNELS_LIB=$V/mf32/libljs_kernels.so python bench.py --batch-per-gpu 8 --steps 20 --warmup 5
done
step $O/l8_1.txt timeout -k 10 300 python bench.py --model layer --fp8 --steps 20 --warmup 5
cd /tmp
step $O/prof_l8.log timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof_l8 -o run -- python3 $R/bench.py --model layer --fp8 --steps 20 --warmup 5
cd $R
python scripts/kstats.py $O/prof_l8/run_results.db --steps 86 > $O/l8_kernels.md 2>&1
for f in $O/[bl]*_*.txt; do echo "$(basename $f) $(grep -o '"ms_per_step": [0-9.]*' $f)"; done > $O/lines.txt
echo done
