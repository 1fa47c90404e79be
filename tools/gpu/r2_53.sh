#!/bin/bash
# DP merge path with the host-segment gather (DIE_DP_COMM=host, no RCCL communicator) vs RCCL device
# gather, solo and plain worker; GPU DP tests for all three paths first.
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2_53
mkdir -p $O
export DIE_TUNE_CACHE=$O/tune.json
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_dp.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { grep -E "Error|assert|FAIL" $O/tests.log | cut -c1-300 | tail -20; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() {
  n=$1; shift
  timeout -k 10 400 python bench.py --steps 20 --warmup 5 "$@" > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  python -c "import json;d=json.load(open('$O/$n.json'));print('$n',round(d['value']),d['p50_ms'],d['p99_ms'],d.get('avg_batch'),d.get('avg_dp_batch'),d.get('dp_backend'),d.get('stages_us'))"
}
DIE_DP_FORCE_MERGE=1 DIE_DP_COMM=host run merge_host --mode dp
DIE_DP_FORCE_MERGE=1 run merge_rccl --mode dp
run http --mode http
DIE_DP_FORCE_MERGE=1 DIE_DP_COMM=host run merge_host2 --mode dp
DIE_DP_FORCE_MERGE=1 run merge_rccl2 --mode dp
run solo --mode dp
