#!/bin/bash
# round 2 start: GPU tests, driver-shaped bench, long bench, rocprof kernel stats of the serving path
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2_01
mkdir -p $O
export DIE_TUNE_CACHE=$O/tune.json
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/b20.json 2> $O/b20.err || exit 1
timeout -k 10 300 python bench.py --steps 400 --warmup 30 > $O/b400.json 2> $O/b400.err || exit 1
for f in b20 b400; do python -c "import json;d=json.load(open('$O/$f.json'));print('$f',round(d['value']),d['p50_ms'],d['p99_ms'],round(d['avg_batch'],1),d['stages_us'])"; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 200 --warmup 20 > $O/prof.log 2>&1 || exit 1
find $O/prof -name '*kernel_stats.csv' | head -3
