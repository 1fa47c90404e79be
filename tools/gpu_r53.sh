#!/bin/bash
# per-op A/B: pre-activation on load vs dual store, batch 24
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r53
mkdir -p $O
export DIE_TUNE_CACHE=$O/tune.json
timeout -k 10 300 python tools/op_profile.py --arch resnet50 --batch 24 --out $O/ops_preact > /dev/null 2>&1 || exit 1
DIE_NO_BN_ON_LOAD=1 timeout -k 10 300 python tools/op_profile.py --arch resnet50 --batch 24 --out $O/ops_dual > /dev/null 2>&1 || exit 1
head -3 $O/ops_preact.md | tail -1; head -3 $O/ops_dual.md | tail -1
