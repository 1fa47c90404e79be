#!/bin/bash
# current-state profiles: per-op at the serving batch (20) and 32, rocprofv3 kernel stats of the headline
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r55
mkdir -p $O
export DIE_TUNE_CACHE=$O/tune.json
timeout -k 10 300 python tools/op_profile.py --arch resnet50 --batch 20 --out $O/ops_rn50_b20 > /dev/null 2>&1 || exit 1
timeout -k 10 300 python tools/op_profile.py --arch resnet50 --batch 32 --out $O/ops_rn50_b32 > /dev/null 2>&1 || exit 1
head -3 $O/ops_rn50_b20.md | tail -1; head -3 $O/ops_rn50_b32.md | tail -1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 600 --warmup 30 > $O/prof_bench.json 2> $O/prof_bench.err || exit 1
find $O/prof -name "*kernel_stats.csv" | head -3
