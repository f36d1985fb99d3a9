set -e
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r2f8t.txt
: > $o
for t in 1282 1283 2562 2563; do
  for m in qout qmask; do timeout -k 10 60 python scripts/fp8_one.py 2560 640 $t 50 $m 2>&1 | grep -v amdgpu.ids >> $o; done
  for m in plain res; do timeout -k 10 60 python scripts/fp8_one.py 640 2560 $t 50 $m 2>&1 | grep -v amdgpu.ids >> $o; done
done
