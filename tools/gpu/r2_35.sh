#!/bin/bash
# Parse pool (auto) vs parse on reactors (0): A/B twice, fp32 headline.
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2_35
mkdir -p $O
export DIE_TUNE_CACHE=$O/tune.json
cd $R
for p in 8 4 8 4; do
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --parse-threads $p > $O/p$p.json 2> $O/p$p.err || { tail -20 $O/p$p.err; exit 1; }
python -c "import json;d=json.load(open('$O/p$p.json'));print('parse $p',round(d['value']),d['p50_ms'],d['p99_ms'],d.get('avg_batch'),d.get('stages_us'),round(d.get('direct_worker',{}).get('rps_this_rank',0)))"
done
