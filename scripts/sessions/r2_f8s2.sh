set -e
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r2fs2.txt
: > $o
for t in 1282 2563; do
  for m in plain relu qonly qout; do timeout -k 10 60 python scripts/fp8_one.py 2560 640 $t 50 $m 2>&1 | grep -v amdgpu.ids >> $o; done
done
for t in 1282 2561; do
timeout -k 10 60 python scripts/gemm_one.py ffup $t 1 50 2>&1 | grep -v amdgpu.ids >> $o || true
done
