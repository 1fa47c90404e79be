#!/bin/bash
# DP solo without a communicator (default now): GPU DP tests, dp vs http, then the forced merge path
# (RCCL communicator formed) with per-thread CPU samples taken while it serves, to name the threads
# that cost the host path.
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2_44
mkdir -p $O
export DIE_TUNE_CACHE=$O/tune.json
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_dp.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { grep -E "Error|assert|FAIL" $O/tests.log | cut -c1-300 | tail -20; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() {
  n=$1; shift
  timeout -k 10 400 python bench.py --steps 20 --warmup 5 "$@" > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  python -c "import json;d=json.load(open('$O/$n.json'));print('$n',round(d['value']),d['p50_ms'],d['p99_ms'],d.get('avg_batch'),d.get('avg_dp_batch'),d.get('dp_backend'),d.get('stages_us'))"
}
run dp --mode dp
run http --mode http
# merge path with thread sampling: a long run (60 steps) so the samples land in the timed phase
DIE_DP_FORCE_MERGE=1 timeout -k 10 400 python bench.py --steps 80 --warmup 5 --mode dp --no-direct > $O/dp_merge.json 2> $O/dp_merge.err &
P=$!
for i in $(seq 1 12); do
  sleep 2
  kill -0 $P 2>/dev/null || break
  echo "=== sample $i" >> $O/threads.txt
  top -H -b -n 1 -d 0.5 -p $P 2>&1 | head -30 >> $O/threads.txt || true
done
wait $P || { tail -20 $O/dp_merge.err; exit 1; }
python -c "import json;d=json.load(open('$O/dp_merge.json'));print('dp_merge',round(d['value']),d['p50_ms'],d['p99_ms'],d.get('avg_dp_batch'),d.get('dp_backend'))"
