#!/bin/bash
# ViT-B/16 per-op device time, fp32 (split) vs bf16, batch 32.
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2_36
mkdir -p $O
export DIE_TUNE_CACHE=$O/tune.json
cd $R
for P in fp32 bf16; do
  timeout -k 10 400 python -u tools/op_profile.py --arch vit_b16 --batch 32 --precision $P --out $O/ops_vit_${P}_b32.md > $O/ops_$P.log 2>&1 || { tail -20 $O/ops_$P.log; exit 1; }
  sed -n 3p $O/ops_vit_${P}_b32.md*
done
