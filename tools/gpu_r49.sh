#!/bin/bash
# packed early upload + pacing; live batch on/off
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r49
mkdir -p $O
export DIE_TUNE_CACHE=$O/tune.json
timeout -k 10 600 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_engine.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit 1
tail -1 $O/tests.log
i=0
for cfg in "--stage-slots -1" "" "--stage-slots -1" "" "--stage-slots -1" ""; do
  i=$((i+1))
  l=1; a=$cfg
  case "$cfg" in *LIVE0*) l=0; a=${cfg%LIVE0};; esac
  DIE_LIVE_BATCH=$l timeout -k 10 300 python bench.py --steps 1500 --warmup 30 $a > $O/b$i.json 2> $O/b$i.err || exit 1
  echo "b$i [$cfg] $(python -c "import json,sys;d=json.load(open('$O/b$i.json'));print(round(d['value']),d['p50_ms'],d['p99_ms'],round(d['avg_batch'],1),round(d['device_ms_per_batch'],3),round(d.get('pace_lead_ms'),3),d.get('staged_uploads'),d.get('staging_diag',{}).get('staged_not_ready_at_submit'))")"
done
