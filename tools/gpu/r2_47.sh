#!/bin/bash
# Completion wait: hipEventSynchronize (spins a CPU) vs sleep-poll at 20 / 50 us, headline bench
# (gateway + worker) interleaved; runtime env and thread CPU of the 50 us run recorded.
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2_47
mkdir -p $O
export DIE_TUNE_CACHE=$O/tune.json
cd $R
env | grep -E "^(HSA|HIP|ROC|AMD|GPU)_" | sort > $O/env.txt || true
run() {
  n=$1; shift
  timeout -k 10 400 python bench.py --steps 20 --warmup 5 "$@" > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  python -c "import json;d=json.load(open('$O/$n.json'));print('$n',round(d['value']),d['p50_ms'],d['p99_ms'],d.get('avg_batch'),d.get('cpu_us_per_request'),d.get('direct_worker',{}).get('rps_this_rank'),d.get('stages_us'))"
}
run sync
DIE_COMPLETION_POLL_US=50 run poll50
DIE_COMPLETION_POLL_US=20 run poll20
run sync2
DIE_COMPLETION_POLL_US=50 run poll50b
DIE_COMPLETION_POLL_US=20 run poll20b
