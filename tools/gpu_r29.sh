#!/bin/bash
# copy-stream / HW-queue A/B for early upload
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r29
mkdir -p $O
timeout -k 10 300 python bench.py --steps 30 --warmup 2 > $O/warm.json 2> $O/warm.err || exit 1
i=0
for cfg in "2 0 2 4" "2 -1 1 4" "2 -1 2 8" "2 0 1 4" "1 -1 1 4" "2 -1 2 4"; do
  set -- $cfg
  i=$((i+1))
  DIE_COPY_STREAMS=$3 GPU_MAX_HW_QUEUES=$4 timeout -k 10 240 python bench.py --steps 300 --warmup 10 --pipeline-depth $1 --stage-slots $2 > $O/b${i}_d$1_s$2_c$3_q$4.json 2> $O/b${i}.err || exit 1
done
echo done
