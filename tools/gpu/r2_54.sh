#!/bin/bash
# Final round-end rehearsal of the committed tree (host-gather DP option in): full GPU suite, smoke(), default bench twice.
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2_54
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { grep -E "Error|assert|FAIL" $O/tests.log | cut -c1-300 | tail -20; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_default.json'));print('default',round(d['value']),d['p50_ms'],d['p99_ms'],d.get('avg_batch'),d.get('worker_init_s'),d['steps'],d['warmup'],d['config'])"
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench_20.json 2> $O/bench_20.err || { tail -20 $O/bench_20.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_20.json'));print('steps20',round(d['value']),d['p50_ms'],d['p99_ms'],d.get('avg_batch'),d.get('worker_init_s'))"
