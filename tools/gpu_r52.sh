#!/bin/bash
# pre-activation on load (no dual stores): numerics, forward A/B, headline A/B
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r52
mkdir -p $O
export DIE_TUNE_CACHE=$O/tune.json
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit 1
tail -1 $O/tests.log
for B in 16 24 32; do
  for n in 0 1; do
    if [ $n = 1 ]; then export DIE_NO_BN_ON_LOAD=1; else unset DIE_NO_BN_ON_LOAD; fi
    timeout -k 10 300 python bench.py --mode engine --batch $B --steps 300 --warmup 10 > $O/e${B}_$n.json 2> $O/e${B}_$n.err || exit 1
    python -c "import json;a=json.load(open('$O/e${B}_$n.json'));print('engine B=$B no_preact=$n dev ms',round(a['device_ms_per_batch'],4))"
  done
done
unset DIE_NO_BN_ON_LOAD
i=0
for n in 0 1 0 1; do
  i=$((i+1))
  if [ $n = 1 ]; then export DIE_NO_BN_ON_LOAD=1; else unset DIE_NO_BN_ON_LOAD; fi
  timeout -k 10 300 python bench.py --steps 1500 --warmup 30 > $O/b$i.json 2> $O/b$i.err || exit 1
  echo "b$i [no_preact=$n] $(python -c "import json,sys;d=json.load(open('$O/b$i.json'));print(round(d['value']),d['p50_ms'],d['p99_ms'],round(d['avg_batch'],1),round(d['device_ms_per_batch'],3),round(d.get('pace_lead_ms'),3))")"
done
