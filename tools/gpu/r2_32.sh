#!/bin/bash
# Pipeline depth 4 vs 3 with the fine buckets (A/B twice).
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2_32
mkdir -p $O
export DIE_TUNE_CACHE=$O/tune.json
cd $R
for d in 4 3 4 3; do
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --pipeline-depth $d > $O/d$d.json 2> $O/d$d.err || { tail -20 $O/d$d.err; exit 1; }
python -c "import json;d=json.load(open('$O/d$d.json'));print('depth $d',round(d['value']),d['p50_ms'],d['p99_ms'],d.get('avg_batch'),d.get('device_ms_per_batch'),round(d.get('direct_worker',{}).get('rps_this_rank',0)))"
done
