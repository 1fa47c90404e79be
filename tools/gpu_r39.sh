#!/bin/bash
# kernel trace of the serving path: bubbles inside the forward graph
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r39
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o prof --output-format csv -- python3 bench.py --steps 300 --warmup 10 > $O/bench.json 2> $O/bench.err || exit 1
f=$(find $O/prof -name '*kernel_trace.csv' | head -1)
python3 tools/graph_gaps.py $f --first stem7x7 > $O/gaps.txt && cat $O/gaps.txt
python3 tools/graph_gaps.py $f --first stem7x7 --last 2000 > $O/gaps_all.txt
s=$(find $O/prof -name '*kernel_stats.csv' | head -1); cp $s $O/kernel_stats.csv; gzip -c $f > $O/kernel_trace.csv.gz; rm -rf $O/prof
