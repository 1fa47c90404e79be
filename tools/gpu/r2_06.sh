#!/bin/bash
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2_06
mkdir -p $O
export DIE_TUNE_CACHE=$O/tune.json
timeout -k 10 120 python tools/dbg_stem.py 2>&1 | grep -v amdgpu.ids
summ() { python -c "import json;d=json.load(open('$1'));print('$2',round(d['value']),d['dtype'],'p50',round(d['p50_ms'],2),'p99',round(d['p99_ms'],2),'avgB',round(d['avg_batch'],1),'cpu',d['cpu_us_per_request'],'dev',d.get('device_ms_per_batch'),'direct',{k:v for k,v in d.get('direct_worker',{}).items()})"; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/fp32.json 2> $O/fp32.err || { tail -20 $O/fp32.err; exit 1; }
summ $O/fp32.json fp32
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --precision bf16 > $O/bf16.json 2> $O/bf16.err || { tail -20 $O/bf16.err; exit 1; }
summ $O/bf16.json bf16
