#!/bin/bash
# PREP (decode + input prep) on the copy stream, overlapping the previous MAIN
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r32
mkdir -p $O
timeout -k 10 300 python bench.py --steps 30 --warmup 2 > $O/warm.json 2> $O/warm.err || exit 1
i=0
for cfg in "1 -1" "2 -1" "1 0" "2 0" "1 -1" "2 -1"; do
  set -- $cfg
  i=$((i+1))
  timeout -k 10 240 python bench.py --steps 300 --warmup 10 --pipeline-depth $1 --stage-slots $2 > $O/b${i}_d$1_s$2.json 2> $O/b${i}.err || exit 1
done
echo done
