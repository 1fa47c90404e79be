#!/bin/bash
# NUMA binding A/B + engine-only forward at buckets
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r40
mkdir -p $O
i=0
for cfg in "" "--no-numa" "" "--no-numa" "" "--no-numa"; do
  i=$((i+1))
  timeout -k 10 200 python bench.py --steps 300 --warmup 10 $cfg > $O/b$i.json 2> $O/b$i.err || exit 1
  echo "b$i [$cfg] $(python -c "import json,sys;d=json.load(open('$O/b$i.json'));print(round(d['value']),d['p50_ms'],d['p99_ms'],round(d['avg_batch'],1),round(d['device_ms_per_batch'],3),d.get('pace_lead_ms'),d.get('numa'))")" >> $O/summary.txt
done
cat $O/summary.txt
