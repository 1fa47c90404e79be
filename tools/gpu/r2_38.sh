#!/bin/bash
# Re-entry check of a freshly rebuilt tree: full GPU suite, smoke(), default bench, then DP world=1
# vs plain worker with the whole result documents kept (stage times for the DP overhead hunt).
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2_38
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { grep -E "Error|assert|FAIL" $O/tests.log | cut -c1-300 | tail -20; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_default.json'));print('default',round(d['value']),d['p50_ms'],d['p99_ms'],d.get('avg_batch'),d.get('worker_init_s'),d['steps'],d['warmup'])"
for m in dp http; do
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --mode $m > $O/$m.json 2> $O/$m.err || { tail -20 $O/$m.err; exit 1; }
python -c "import json;d=json.load(open('$O/$m.json'));print('$m',round(d['value']),d['p50_ms'],d['p99_ms'],d.get('avg_batch'),d.get('avg_dp_batch'),d.get('device_ms_per_batch'),d.get('gpu_gap_ms_per_batch'),d.get('stages_us'))"
done
