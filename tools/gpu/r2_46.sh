#!/bin/bash
# Named native threads: per-thread CPU samples of the plain worker (http mode) and of the DP merge
# path (RCCL communicator formed) while they serve; the unnamed busy threads are the runtime's.
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2_46
mkdir -p $O
export DIE_TUNE_CACHE=$O/tune.json
cd $R
sample() {
  n=$1; shift
  timeout -k 10 300 python bench.py --steps 300 --warmup 5 --no-direct "$@" > $O/$n.json 2> $O/$n.err &
  P=$!
  for i in $(seq 1 30); do
    sleep 1.5
    kill -0 $P 2>/dev/null || break
    for c in $(pgrep -P $P); do
      echo "=== $n sample $i pid $c" >> $O/threads_$n.txt
      top -H -b -n 1 -d 0.5 -p $c 2>&1 | sed -n '7,24p' >> $O/threads_$n.txt || true
    done
  done
  wait $P || { tail -20 $O/$n.err; exit 1; }
  python -c "import json;d=json.load(open('$O/$n.json'));print('$n',round(d['value']),d['p50_ms'],d.get('dp_backend'))"
}
sample http --mode http
DIE_DP_FORCE_MERGE=1 sample dp_merge --mode dp
