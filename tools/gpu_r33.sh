#!/bin/bash
# two batches executing concurrently (per-executor arenas) vs one
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r33
mkdir -p $O
timeout -k 10 600 python -m pytest tests/test_gpu_decode.py tests/test_gpu_engine.py tests/test_gpu_dp.py tests/test_gpu_transformer.py -x -q > $O/tests.log 2>&1 || exit 1
i=0
for cfg in "2 1" "2 2" "3 2" "4 2" "2 1" "2 2"; do
  set -- $cfg
  i=$((i+1))
  timeout -k 10 240 python bench.py --steps 300 --warmup 10 --pipeline-depth $1 --exec-streams $2 > $O/b${i}_d$1_e$2.json 2> $O/b${i}.err || exit 1
done
echo done
