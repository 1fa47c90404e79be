#!/bin/bash
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2_09
mkdir -p $O
export DIE_TUNE_CACHE=$O/tune.json
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread -s > $O/tests.log 2>&1 || { grep -E "CONFIG3|Error|assert|FAIL" $O/tests.log | cut -c1-400 | tail -30; tail -5 $O/tests.log; exit 1; }
grep -E "CONFIG3" $O/tests.log | cut -c1-700
tail -2 $O/tests.log
summ() { python -c "import json;d=json.load(open('$1'));print('$2',round(d['value']),d['dtype'],'p50',round(d['p50_ms'],2),'p99',round(d['p99_ms'],2),d.get('avg_batch'),d.get('gateway',{}).get('shm_forwards'),d.get('dp_batches_rank0'))"; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/fp32.json 2> $O/fp32.err || { tail -20 $O/fp32.err; exit 1; }
summ $O/fp32.json fp32
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --mode dp > $O/dp1.json 2> $O/dp1.err || { tail -20 $O/dp1.err; exit 1; }
summ $O/dp1.json dp1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --mode http > $O/http.json 2> $O/http.err || { tail -20 $O/http.err; exit 1; }
summ $O/http.json http
