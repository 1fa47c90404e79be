set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r7
mkdir -p $O
timeout -k 10 300 python -m pytest tests/test_gpu_decode.py -q > $O/dec.log 2>&1 && \
timeout -k 10 300 python tools/decode_bench.py > $O/dec_bench.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 200 --warmup 5 > $O/bench.log 2>&1
echo "exit=$?"
