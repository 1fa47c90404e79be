#!/bin/bash
# staging A/B: compute + 2 copy streams (D2H on the compute stream)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r24
mkdir -p $O
timeout -k 10 600 python -m pytest tests/test_gpu_decode.py tests/test_gpu_engine.py tests/test_gpu_dp.py -x -q > $O/tests.log 2>&1 || exit 1
for cfg in "2 -1 4" "2 0 4" "1 -1 4" "3 -1 4"; do
  set -- $cfg
  GPU_MAX_HW_QUEUES=$3 timeout -k 10 240 python bench.py --steps 300 --warmup 10 --pipeline-depth $1 --stage-slots $2 > $O/bench_d$1_s$2_q$3.json 2> $O/bench_d$1_s$2_q$3.err || exit 1
done
echo done
