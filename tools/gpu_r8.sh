set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r8
mkdir -p $O
timeout -k 10 300 python -m pytest tests/test_gpu_dp.py -x -q > $O/dp.log 2>&1 && \
timeout -k 10 300 python bench.py --mode dp --steps 100 --warmup 5 > $O/bench_dp1.log 2>&1 && \
timeout -k 10 600 python -m pytest tests/ -q -m gpu > $O/all_gpu.log 2>&1
echo "exit=$?"
