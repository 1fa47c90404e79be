#!/bin/bash
# Fused NCHW stem (input prep in the stem's patch loader): kernel tests, engine numerics, per-op, bench.
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2_14
mkdir -p $O
export DIE_TUNE_CACHE=$O/tune.json
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_fp32.py tests/test_gpu_dp.py tests/test_gpu_engine.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -u tools/op_profile.py --arch resnet50 --batch 32 --precision fp32 --out $O/ops_fp32_b32.md > $O/ops.log 2>&1 || { tail -20 $O/ops.log; exit 1; }
head -4 $O/ops_fp32_b32.md.md; sed -n 7,9p $O/ops_fp32_b32.md.md
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/fp32.json 2> $O/fp32.err || { tail -20 $O/fp32.err; exit 1; }
python -c "import json;d=json.load(open('$O/fp32.json'));print('fp32',round(d['value']),d['p50_ms'],d['p99_ms'],d.get('direct_worker'),d.get('worker_init_s'))"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --mode dp > $O/dp1.json 2> $O/dp1.err || { tail -20 $O/dp1.err; exit 1; }
python -c "import json;d=json.load(open('$O/dp1.json'));print('dp1',round(d['value']),d['p50_ms'],d.get('avg_dp_batch'),d.get('device_ms_per_batch'),d.get('gpu_gap_ms_per_batch'),d.get('stages_us'))"
