#!/bin/bash
# early text upload + finer buckets: tests, then A/B of staging and pipeline depth on the headline
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r20
mkdir -p $O
timeout -k 10 600 python -m pytest tests/test_gpu_decode.py tests/test_gpu_engine.py -x -q > $O/tests.log 2>&1 || exit 1
for cfg in "2 -1" "2 0" "1 -1" "1 0"; do
  set -- $cfg
  timeout -k 10 240 python bench.py --steps 300 --warmup 10 --pipeline-depth $1 --stage-slots $2 > $O/bench_d$1_s$2.json 2> $O/bench_d$1_s$2.err || exit 1
done
echo done
