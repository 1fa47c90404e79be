set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r5
mkdir -p $O
timeout -k 10 600 python -m pytest tests/test_gpu_decode.py -q > $O/dec.log 2>&1 && \
timeout -k 10 600 python -m pytest tests/test_gpu_engine.py tests/test_gpu_transformer.py -x -q > $O/eng.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 200 --warmup 5 > $O/bench.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 200 --warmup 5 --no-device-decode > $O/bench_host.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 200 --warmup 5 --connections 96 > $O/bench_c96.log 2>&1 && \
timeout -k 10 300 python bench.py --arch vit_b16 --steps 100 --warmup 3 > $O/bench_vit.log 2>&1
echo "exit=$?"
