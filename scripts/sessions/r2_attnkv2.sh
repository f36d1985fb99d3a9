set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
o=gpurun_out/r2attnkv2.txt
: > $o
for i in 1 2; do
for lib in old new; do
  if [ $lib = old ]; then export LJS_KERNELS_LIB=$PWD/learning_jax_sharding_amd/_lib/libljs_kernels_old.so; else unset LJS_KERNELS_LIB; fi
  echo "$lib $(timeout -k 10 120 python scripts/attn_time.py 2>&1 | tail -1)" >> $o
  echo "$lib $(timeout -k 10 120 python scripts/attn_time.py 8 256 8 2>&1 | tail -1)" >> $o
done
done
unset LJS_KERNELS_LIB
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r2kv_b64 -o prof -- python bench.py --steps 20 --warmup 5 > gpurun_out/r2kv_b64.log 2>&1
