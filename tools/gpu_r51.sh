#!/bin/bash
# pacing deadline experiment: dispatch later than the copy lead (trade GPU idle for batch size)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r51
mkdir -p $O
export DIE_TUNE_CACHE=$O/tune.json
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit 1
tail -1 $O/tests.log
i=0
for sc in 1 0.6 0.3 0 1 0.6 0.3 0; do
  i=$((i+1))
  DIE_PACE_LEAD_SCALE=$sc timeout -k 10 300 python bench.py --steps 1500 --warmup 30 > $O/b$i.json 2> $O/b$i.err || exit 1
  echo "b$i [scale=$sc] $(python -c "import json,sys;d=json.load(open('$O/b$i.json'));print(round(d['value']),d['p50_ms'],d['p99_ms'],round(d['avg_batch'],1),round(d['device_ms_per_batch'],3),round(d.get('pace_lead_ms'),3),round(d['copy_wait_ms_per_batch'],3))")"
done
