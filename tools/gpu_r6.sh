set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r6
mkdir -p $O
timeout -k 10 300 python tools/op_profile.py --arch resnet50 --batch 32 --out $O/ops_rn50_b32 > $O/ops_rn50.log 2>&1 && \
timeout -k 10 300 python tools/op_profile.py --arch vit_b16 --batch 32 --out $O/ops_vit_b32 > $O/ops_vit.log 2>&1 && \
timeout -k 10 300 python tools/op_profile.py --arch resnet50 --batch 16 --out $O/ops_rn50_b16 > $O/ops_rn50_16.log 2>&1
echo "exit=$?"
