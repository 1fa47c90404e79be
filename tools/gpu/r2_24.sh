#!/bin/bash
# Pacing margin also adapts to pre-submit GPU gaps: A/B with DIE_PACE_GAP=0/1, twice.
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2_24
mkdir -p $O
export DIE_TUNE_CACHE=$O/tune.json
cd $R
for g in 1 0 1 0; do
DIE_PACE_GAP=$g timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/g$g.json 2> $O/g$g.err || { tail -20 $O/g$g.err; exit 1; }
python -c "import json;d=json.load(open('$O/g$g.json'));print('gapadapt $g',round(d['value']),d['p50_ms'],d['p99_ms'],d.get('avg_batch'),d.get('device_ms_per_batch'),d.get('gpu_gap_ms_per_batch'),d.get('pace_lead_ms'),round(d.get('direct_worker',{}).get('rps_this_rank',0)))"
done
