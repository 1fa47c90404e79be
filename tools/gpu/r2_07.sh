#!/bin/bash
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2_07
mkdir -p $O
export DIE_TUNE_CACHE=$O/tune.json
summ() { python -c "import json;d=json.load(open('$1'));print('$2',round(d['value']),d['dtype'],'p50',round(d['p50_ms'],2),'p99',round(d['p99_ms'],2),'avgB',round(d['avg_batch'],1),'cpu',d['cpu_us_per_request'],'gw',d.get('gateway'),'direct',{k:v for k,v in d.get('direct_worker',{}).items()})"; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/fp32.json 2> $O/fp32.err || { tail -20 $O/fp32.err; exit 1; }
summ $O/fp32.json fp32
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --precision bf16 > $O/bf16.json 2> $O/bf16.err || { tail -20 $O/bf16.err; exit 1; }
summ $O/bf16.json bf16
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-local-shm > $O/fp32_noshm.json 2> $O/fp32_noshm.err || { tail -20 $O/fp32_noshm.err; exit 1; }
summ $O/fp32_noshm.json fp32_noshm
timeout -k 10 600 python -u -m pytest tests/test_gpu_fp32.py -x -q --timeout 300 --timeout-method thread > $O/fp32.log 2>&1 || { tail -40 $O/fp32.log; exit 1; }
tail -1 $O/fp32.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_cluster.py -x -v -s --timeout 300 --timeout-method thread > $O/cluster.log 2>&1 || { tail -40 $O/cluster.log; exit 1; }
grep -E "CONFIG3|passed|failed" $O/cluster.log | cut -c1-600
