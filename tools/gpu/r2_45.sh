#!/bin/bash
# RCCL host cost: merge path (RCCL comm formed) with the init's CPU-mask change undone, vs http;
# then per-thread CPU samples of a long merge-path run (the python child, not the timeout wrapper).
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2_45
mkdir -p $O
export DIE_TUNE_CACHE=$O/tune.json
cd $R
run() {
  n=$1; shift
  timeout -k 10 400 python bench.py --steps 20 --warmup 5 "$@" > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  python -c "import json;d=json.load(open('$O/$n.json'));print('$n',round(d['value']),d['p50_ms'],d['p99_ms'],d.get('avg_batch'),d.get('avg_dp_batch'),d.get('dp_backend'),d.get('dp_affinity_restores'),d.get('host_cpus'),d.get('stages_us'))"
}
DIE_DP_FORCE_MERGE=1 run dp_merge --mode dp
run http --mode http
DIE_DP_FORCE_MERGE=1 run dp_merge2 --mode dp
run dp --mode dp
DIE_DP_FORCE_MERGE=1 timeout -k 10 300 python bench.py --steps 400 --warmup 5 --mode dp --no-direct > $O/dp_long.json 2> $O/dp_long.err &
P=$!
for i in $(seq 1 40); do
  sleep 1.5
  kill -0 $P 2>/dev/null || break
  C=$(pgrep -P $P | tr '\n' ' ')
  for c in $C; do
    echo "=== sample $i pid $c" >> $O/threads.txt
    top -H -b -n 1 -d 0.5 -p $c 2>&1 | sed -n '7,30p' >> $O/threads.txt || true
  done
done
wait $P || { tail -20 $O/dp_long.err; exit 1; }
python -c "import json;d=json.load(open('$O/dp_long.json'));print('dp_long',round(d['value']),d['p50_ms'],d.get('dp_backend'),d.get('dp_affinity_restores'))"
