set -e
cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python bench.py --steps 100 --warmup 10 > gpurun_out/m_train64.log 2>&1
timeout -k 10 200 python bench.py --mode fwd --steps 100 --warmup 10 > gpurun_out/m_fwd64.log 2>&1
timeout -k 10 200 python bench.py --batch-per-gpu 8 --steps 200 --warmup 20 > gpurun_out/m_train8.log 2>&1
timeout -k 10 200 python bench.py --batch-per-gpu 8 --mode fwd --steps 200 --warmup 20 > gpurun_out/m_fwd8.log 2>&1
LJS_PLATFORM=gpu timeout -k 10 300 python cases/case6_attention.py > gpurun_out/m_case6.log 2>&1
