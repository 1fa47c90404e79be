#!/bin/bash
# Worker reactors: auto (16) vs 32, three interleaved pairs (second box).
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2_51
mkdir -p $O
export DIE_TUNE_CACHE=$O/tune.json
cd $R
run() {
  n=$1; shift
  timeout -k 10 400 python bench.py --steps 20 --warmup 5 "$@" > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  python -c "import json;d=json.load(open('$O/$n.json'));print('$n',round(d['value']),d['p50_ms'],d['p99_ms'],d.get('avg_batch'),d.get('cpu_us_per_request'),round(d.get('direct_worker',{}).get('rps_this_rank',0)),d.get('stages_us'))"
}
run auto
run w32 --worker-http-threads 32
run auto2
run w32b --worker-http-threads 32
run auto3
run w32c --worker-http-threads 32
