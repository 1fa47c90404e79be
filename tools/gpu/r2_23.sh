#!/bin/bash
# Two concurrent executors (exec_streams 2) vs one, fp32 headline.
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2_23
mkdir -p $O
export DIE_TUNE_CACHE=$O/tune.json
cd $R
for cfg in "1 3" "2 4" "2 3" "1 3"; do
set -- $cfg
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --exec-streams $1 --pipeline-depth $2 > $O/e$1_d$2.json 2> $O/e$1_d$2.err || { tail -20 $O/e$1_d$2.err; exit 1; }
python -c "import json;d=json.load(open('$O/e$1_d$2.json'));print('exec $1 depth $2',round(d['value']),d['p50_ms'],d['p99_ms'],d.get('avg_batch'),d.get('device_ms_per_batch'),round(d.get('direct_worker',{}).get('rps_this_rank',0)))"
done
