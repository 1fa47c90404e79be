#!/bin/bash
# DP solo: is the remaining world=1 gap the RCCL communicator's host threads?  dp (solo, RCCL comm
# formed) / dp solo without a communicator / http, interleaved.
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2_43
mkdir -p $O
export DIE_TUNE_CACHE=$O/tune.json
cd $R
run() {
  n=$1; shift
  timeout -k 10 400 python bench.py --steps 20 --warmup 5 "$@" > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  python -c "import json;d=json.load(open('$O/$n.json'));print('$n',round(d['value']),d['p50_ms'],d['p99_ms'],d.get('avg_batch'),d.get('avg_dp_batch'),d.get('stages_us'))"
}
run http --mode http
run dp --mode dp
DIE_DP_SOLO_NO_COMM=1 run dp_nocomm --mode dp
run http2 --mode http
DIE_DP_SOLO_NO_COMM=1 run dp_nocomm2 --mode dp
run dp2 --mode dp
