#!/bin/bash
# XCD-aware conv block mapping: numerics, conv sweep at b16/b32, headline bench
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r42
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit 1
tail -2 $O/tests.log
timeout -k 10 300 python tools/conv_bench.py --batch 16 --json $O/conv_b16.json --md $O/conv_b16.md > $O/b16.log 2>&1 || exit 1
timeout -k 10 300 python tools/conv_bench.py --batch 32 --json $O/conv_b32.json --md $O/conv_b32.md > $O/b32.log 2>&1 || exit 1
head -4 $O/conv_b16.md | tail -1; head -4 $O/conv_b32.md | tail -1
for i in 1 2; do
timeout -k 10 200 python bench.py --steps 400 --warmup 20 > $O/bench$i.json 2> $O/bench$i.err || exit 1
python -c "import json,sys;d=json.load(open('$O/bench$i.json'));print(round(d['value']),d['p50_ms'],d['p99_ms'],round(d['avg_batch'],1),round(d['device_ms_per_batch'],3),d.get('pace_lead_ms'))"
done
