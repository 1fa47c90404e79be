set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r15
mkdir -p $O
timeout -k 10 300 python -m pytest tests/test_gpu_transformer.py -x -q > $O/tf.log 2>&1 && \
timeout -k 10 300 python tools/op_profile.py --arch vit_b16 --batch 32 --out $O/ops_vit_b32 > $O/ops.log 2>&1
echo "exit=$?"
