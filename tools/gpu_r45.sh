#!/bin/bash
# PREP in line on the compute stream vs beside the previous MAIN (copy stream)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r45
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_engine.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit 1
DIE_PREP_ON_COMPUTE=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py -x -q --timeout 120 --timeout-method thread > $O/tests_poc.log 2>&1 || exit 1
tail -1 $O/tests.log $O/tests_poc.log
i=0
for poc in 0 1 0 1 0 1; do
  i=$((i+1))
  DIE_PREP_ON_COMPUTE=$poc timeout -k 10 200 python bench.py --steps 400 --warmup 20 > $O/b$i.json 2> $O/b$i.err || exit 1
  echo "b$i [poc=$poc] $(python -c "import json,sys;d=json.load(open('$O/b$i.json'));print(round(d['value']),d['p50_ms'],d['p99_ms'],round(d['avg_batch'],1),round(d['device_ms_per_batch'],3),round(d.get('pace_lead_ms'),3),round(d['prep_ms_per_batch'],3),round(d['copy_wait_ms_per_batch'],3))")"
done
