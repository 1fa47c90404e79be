#!/bin/bash
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r22
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
GPU_MAX_HW_QUEUES=8 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $O/tr -o t -- python3 bench.py --steps 60 --warmup 5 --pipeline-depth 2 > $O/bench.json 2> $O/bench.err
echo rc=$?
