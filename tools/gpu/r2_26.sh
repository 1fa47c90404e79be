#!/bin/bash
# Finer batch buckets above 16 (20/24/28/32) vs sqrt(2) buckets: A/B twice, plus worker init time.
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2_26
mkdir -p $O
export DIE_TUNE_CACHE=$O/tune.json
cd $R
for c in 0 1 0 1; do
DIE_COARSE_BUCKETS=$c timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/c$c.json 2> $O/c$c.err || { tail -20 $O/c$c.err; exit 1; }
python -c "import json;d=json.load(open('$O/c$c.json'));print('coarse $c',round(d['value']),d['p50_ms'],d['p99_ms'],d.get('avg_batch'),d.get('device_ms_per_batch'),d.get('worker_init_s'),round(d.get('direct_worker',{}).get('rps_this_rank',0)))"
done
