#!/bin/bash
# DP world=1 overhead hunt: leader wait breakdown (pop / slot / pace) with default, unpaced and
# 80-connection clients, plain worker at 80 connections for comparison.
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2_39
mkdir -p $O
export DIE_TUNE_CACHE=$O/tune.json
cd $R
run() {
  n=$1; shift
  timeout -k 10 400 python bench.py --steps 20 --warmup 5 "$@" > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  python -c "import json;d=json.load(open('$O/$n.json'));print('$n',round(d['value']),d['p50_ms'],d['p99_ms'],d.get('avg_batch'),d.get('avg_dp_batch'),d.get('device_ms_per_batch'),d.get('gpu_gap_ms_per_batch'),d.get('pace_lead_ms'),d.get('prep_ms_per_batch'),d.get('leader_wait_ms_per_batch'),d.get('stages_us'))"
}
run dp --mode dp
run http --mode http
run dp_nopace --mode dp --no-pace
run dp_c80 --mode dp --connections 80
run http_c80 --mode http --connections 80
