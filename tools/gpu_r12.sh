set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r12
mkdir -p $O
timeout -k 10 300 python bench.py --steps 300 --warmup 5 > $O/bench.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 300 --warmup 5 --pipeline-depth 3 > $O/bench_d3.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 300 --warmup 5 --pipeline-depth 1 > $O/bench_d1.log 2>&1
echo "exit=$?"
