set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r3e
mkdir -p $O
V=$R/learning_jax_sharding_amd/_lib/variants/pk0/libljs_kernels.so
cd /tmp
for w in fwd bwd; do
  for cfg in "64 256 8" "4 4096 8"; do
    tag=$(echo $w $cfg | tr ' ' '_')
    timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/kt_base_$tag -o run -- python3 $R/scripts/attn_one.py $w $cfg 10 > $O/kt_base_$tag.log 2>&1
    LJS_KERNELS_LIB=$V timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/kt_pk0_$tag -o run -- python3 $R/scripts/attn_one.py $w $cfg 10 > $O/kt_pk0_$tag.log 2>&1
  done
done
cd $R
for i in 1 2; do
  timeout -k 10 200 python bench.py >> $O/b64_base.log 2>&1
  LJS_KERNELS_LIB=$V timeout -k 10 200 python bench.py >> $O/b64_pk0.log 2>&1
  timeout -k 10 200 python bench.py --seq 4096 --batch-per-gpu 4 >> $O/long_base.log 2>&1
  LJS_KERNELS_LIB=$V timeout -k 10 200 python bench.py --seq 4096 --batch-per-gpu 4 >> $O/long_pk0.log 2>&1
done
echo done
