cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r3e
mkdir -p $O
step() { local log=$1; shift; "$@" > "$log" 2>&1; local rc=$?; if [ $rc -ne 0 ]; then echo "rc=$rc: $*" >> $O/rc.log; case $rc in 1|2) ;; *) exit $rc;; esac; fi; }
# A/B of the attention softmax math: packed f32 pairs (base), scalar f32 (pk0, also no SLP
# vectorisation anywhere), packed with SLP off elsewhere (pk1ns)
V0=$R/learning_jax_sharding_amd/_lib/variants/pk0/libljs_kernels.so
V1=$R/learning_jax_sharding_amd/_lib/variants/pk1ns/libljs_kernels.so
step $O/tests_pk0.log env LJS_KERNELS_LIB=$V0 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "attention or attn"
cd /tmp
for w in fwd bwd; do
  for cfg in "64 256 8" "4 4096 8"; do
    tag=$(echo $w $cfg | tr ' ' '_')
    step $O/kt_base_$tag.log timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/kt_base_$tag -o run -- python3 $R/scripts/attn_one.py $w $cfg 10
    step $O/kt_pk0_$tag.log env LJS_KERNELS_LIB=$V0 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/kt_pk0_$tag -o run -- python3 $R/scripts/attn_one.py $w $cfg 10
    step $O/kt_pk1ns_$tag.log env LJS_KERNELS_LIB=$V1 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/kt_pk1ns_$tag -o run -- python3 $R/scripts/attn_one.py $w $cfg 10
  done
done
cd $R
for i in 1 2; do
  step $O/b64_base_$i.log timeout -k 10 200 python bench.py
  step $O/b64_pk0_$i.log env LJS_KERNELS_LIB=$V0 timeout -k 10 200 python bench.py
  step $O/b64_pk1ns_$i.log env LJS_KERNELS_LIB=$V1 timeout -k 10 200 python bench.py
  step $O/long_base_$i.log timeout -k 10 200 python bench.py --seq 4096 --batch-per-gpu 4
  step $O/long_pk0_$i.log env LJS_KERNELS_LIB=$V0 timeout -k 10 200 python bench.py --seq 4096 --batch-per-gpu 4
done
echo done
