#!/bin/bash
# XCD tile order by real operand bytes: sweeps at B=16/32 fp32, bench depth 2 vs 3 (twice).
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2_19
mkdir -p $O
export DIE_TUNE_CACHE=$O/tune.json
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_fp32.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for B in 16 32; do
timeout -k 10 300 python -u tools/conv_bench.py --batch $B --split --md $O/sweep_fp32_b$B.md > $O/sweep$B.log 2>&1 || { tail -20 $O/sweep$B.log; exit 1; }
tail -1 $O/sweep$B.log
done
for d in 3 2 3 2; do
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --pipeline-depth $d > $O/fp32_d$d.json 2> $O/fp32_d$d.err || { tail -20 $O/fp32_d$d.err; exit 1; }
python -c "import json;d=json.load(open('$O/fp32_d$d.json'));print('depth $d',round(d['value']),d['p50_ms'],d['p99_ms'],d.get('avg_batch'),d.get('device_ms_per_batch'),d.get('gpu_gap_ms_per_batch'),round(d.get('direct_worker',{}).get('rps_this_rank',0)))"
done
