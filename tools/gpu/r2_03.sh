#!/bin/bash
# headline in the new topology: fp32 gateway+worker (driver command), bf16, direct http; op profile fp32
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2_03
mkdir -p $O
export DIE_TUNE_CACHE=$O/tune.json
summ() { python -c "import json;d=json.load(open('$1'));print('$2',round(d['value']),d['dtype'],d['config']['requests'],'p50',round(d['p50_ms'],2),'p99',round(d['p99_ms'],2),'avgB',round(d['avg_batch'],1),'dev',d.get('device_ms_per_batch'),d.get('stages_us'),'direct',d.get('direct_worker'))"; }
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/fp32_gw.json 2> $O/fp32_gw.err || { tail -20 $O/fp32_gw.err; exit 1; }
summ $O/fp32_gw.json fp32_gw
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --precision bf16 > $O/bf16_gw.json 2> $O/bf16_gw.err || { tail -20 $O/bf16_gw.err; exit 1; }
summ $O/bf16_gw.json bf16_gw
timeout -k 10 300 python tools/op_profile.py --arch resnet50 --batch 32 --precision fp32 --out $O/ops_rn50_fp32_b32 > $O/op.log 2>&1 || { tail -20 $O/op.log; exit 1; }
tail -5 $O/ops_rn50_fp32_b32.md
