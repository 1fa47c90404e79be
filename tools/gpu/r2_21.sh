#!/bin/bash
# ViT-B/16 fp32 per-op profile + bench with the reactor-side respond change.
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2_21
mkdir -p $O
export DIE_TUNE_CACHE=$O/tune.json
cd $R
timeout -k 10 400 python -u tools/op_profile.py --arch vit_b16 --batch 32 --precision fp32 --out $O/ops_vit_fp32_b32.md > $O/ops_vit.log 2>&1 || { tail -20 $O/ops_vit.log; exit 1; }
sed -n 3p $O/ops_vit_fp32_b32.md.md; tail -12 $O/ops_vit_fp32_b32.md.md
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/fp32.json 2> $O/fp32.err || { tail -20 $O/fp32.err; exit 1; }
python -c "import json;d=json.load(open('$O/fp32.json'));print('fp32',round(d['value']),d['p50_ms'],d['p99_ms'],d.get('avg_batch'),d.get('stages_us'),round(d.get('direct_worker',{}).get('rps_this_rank',0)))"
