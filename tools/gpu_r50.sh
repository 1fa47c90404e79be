#!/bin/bash
# per-op profiles after cold tuning + live batch; ViT headline
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r50
mkdir -p $O
export DIE_TUNE_CACHE=$O/tune.json
timeout -k 10 300 python tools/op_profile.py --arch resnet50 --batch 16 --out $O/ops_rn50_b16 > /dev/null 2>&1 || exit 1
timeout -k 10 300 python tools/op_profile.py --arch resnet50 --batch 24 --out $O/ops_rn50_b24 > /dev/null 2>&1 || exit 1
timeout -k 10 300 python tools/op_profile.py --arch vit_b16 --batch 32 --out $O/ops_vit_b32 > /dev/null 2>&1 || exit 1
head -3 $O/ops_rn50_b16.md | tail -1; head -3 $O/ops_rn50_b24.md | tail -1; head -3 $O/ops_vit_b32.md | tail -1
timeout -k 10 300 python bench.py --arch vit_b16 --steps 600 --warmup 20 > $O/vit.json 2> $O/vit.err || exit 1
python -c "import json,sys;d=json.load(open('$O/vit.json'));print('vit',round(d['value']),d['p50_ms'],d['p99_ms'],round(d['avg_batch'],1),round(d['device_ms_per_batch'],3),round(d.get('pace_lead_ms'),3))"
