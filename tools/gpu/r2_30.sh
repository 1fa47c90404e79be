#!/bin/bash
# DP: packed text + no 1-rank collectives; dp1 vs http on one box; bucket step 16 vs 8 (A/B).
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2_30
mkdir -p $O
export DIE_TUNE_CACHE=$O/tune.json
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_dp.py tests/test_gpu_decode.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { grep -E "Error|assert|FAIL" $O/tests.log | cut -c1-300 | tail -20; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for m in dp http dp http; do
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --mode $m > $O/$m.json 2> $O/$m.err || { tail -20 $O/$m.err; exit 1; }
python -c "import json;d=json.load(open('$O/$m.json'));print('$m',round(d['value']),d['p50_ms'],d['p99_ms'],d.get('avg_batch'),d.get('avg_dp_batch'),d.get('device_ms_per_batch'),d.get('gpu_gap_ms_per_batch'))"
done
for d in 16 8; do
DIE_BUCKET_DIV=$d timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/div$d.json 2> $O/div$d.err || { tail -20 $O/div$d.err; exit 1; }
python -c "import json;d=json.load(open('$O/div$d.json'));print('div $d',round(d['value']),d['p50_ms'],d['p99_ms'],d.get('avg_batch'),d.get('worker_init_s'))"
done
