#!/bin/bash
# Bucket granularity above 16: every 4 (default) vs every 2 (DIE_BUCKET_DIV=8), A/B twice.
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2_28
mkdir -p $O
export DIE_TUNE_CACHE=$O/tune.json
cd $R
for d in 8 4 8 4; do
DIE_BUCKET_DIV=$d timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/d$d.json 2> $O/d$d.err || { tail -20 $O/d$d.err; exit 1; }
python -c "import json;d=json.load(open('$O/d$d.json'));print('div $d',round(d['value']),d['p50_ms'],d['p99_ms'],d.get('avg_batch'),d.get('device_ms_per_batch'),d.get('worker_init_s'),round(d.get('direct_worker',{}).get('rps_this_rank',0)))"
done
