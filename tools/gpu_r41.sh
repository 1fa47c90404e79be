#!/bin/bash
# model-based pacing lead: A/B vs no pacing
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r41
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_engine.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit 1
i=0
for cfg in "" "--no-pace" "" "--no-pace" "" "--no-pace"; do
  i=$((i+1))
  timeout -k 10 200 python bench.py --steps 400 --warmup 20 $cfg > $O/b$i.json 2> $O/b$i.err || exit 1
  echo "b$i [$cfg] $(python -c "import json,sys;d=json.load(open('$O/b$i.json'));print(round(d['value']),d['p50_ms'],d['p99_ms'],round(d['avg_batch'],1),round(d['device_ms_per_batch'],3),d.get('pace_lead_ms'),d.get('copy_wait_ms_per_batch'),d['stages_us'])")" >> $O/summary.txt
done
cat $O/summary.txt
