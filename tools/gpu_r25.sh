#!/bin/bash
# GPU timelines of the serving loop, staged vs submit-time copies (tune cache warmed first)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r25
mkdir -p $O
timeout -k 10 300 python bench.py --steps 30 --warmup 2 > $O/warm.json 2> $O/warm.err || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for st in -1 0; do
  timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/tr_s$st -o t -- python3 bench.py --steps 100 --warmup 5 --pipeline-depth 2 --stage-slots $st > $O/bench_s$st.json 2> $O/bench_s$st.err || exit 1
done
echo done
