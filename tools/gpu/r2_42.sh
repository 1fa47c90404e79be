#!/bin/bash
# DP world of one = plain local engine + its pinned pool (no arena staging, no gather): GPU DP tests,
# the merge loop forced, same box.
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2_42
mkdir -p $O
export DIE_TUNE_CACHE=$O/tune.json
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_dp.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { grep -E "Error|assert|FAIL" $O/tests.log | cut -c1-300 | tail -20; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() {
  n=$1; shift
  timeout -k 10 400 python bench.py --steps 20 --warmup 5 "$@" > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  python -c "import json;d=json.load(open('$O/$n.json'));print('$n',round(d['value']),d['p50_ms'],d['p99_ms'],d.get('avg_batch'),d.get('avg_dp_batch'),d.get('stages_us'))"
}
run dp --mode dp
run http --mode http
DIE_DP_FORCE_MERGE=1 run dp_merge --mode dp
run dp2 --mode dp
run http2 --mode http
