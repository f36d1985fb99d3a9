# round-6: the MX-fp8 transposed copy by transposing LDS reads (A/B) + fp8 correctness
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r6r
mkdir -p $O
V=$R/learning_jax_sharding_amd/_lib/variants
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; echo "rc=$rc: $*" >> $O/rc.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
step $O/tests.txt timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_gpu_e2e.py -k "fp8 or mx"
step $O/up_new.txt timeout -k 10 300 python scripts/fp8_upproj_probe.py 20
step $O/up_old.txt timeout -k 10 300 env LJS_KERNELS_LIB=$V/qtold/libljs_kernels.so python scripts/fp8_upproj_probe.py 20
for rep in 1 2 3; do
  step $O/l8_new_$rep.txt timeout -k 10 300 python bench.py --model layer --fp8 --steps 20 --warmup 5
  step $O/l8_old_$rep.txt timeout -k 10 300 env LJS_KERNELS_LIB=$V/qtold/libljs_kernels.so python bench.py --model layer --fp8 --steps 20 --warmup 5
done
for f in $O/l8_*.txt; do echo "$(basename $f) $(grep -o '"ms_per_step": [0-9.]*' $f)"; done > $O/lines.txt
echo done
