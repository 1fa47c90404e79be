set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r14
mkdir -p $O
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -x -q > $O/kern.log 2>&1 && \
timeout -k 10 300 python -m pytest tests/test_gpu_engine.py tests/test_gpu_transformer.py -x -q > $O/eng.log 2>&1 && \
timeout -k 10 300 python tools/op_profile.py --arch resnet50 --batch 16 --out $O/ops_rn50_b16 > $O/ops.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 300 --warmup 5 > $O/bench.log 2>&1
echo "exit=$?"
