#!/bin/bash
# Residual prefetch in the glds kernel: tests, expand-conv sweeps (fp32 B=32/16), bench.
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2_25
mkdir -p $O
export DIE_TUNE_CACHE=$O/tune.json
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_fp32.py tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { grep -E "Error|assert|FAIL" $O/tests.log | cut -c1-300 | tail -20; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for B in 32 16; do
timeout -k 10 300 python -u tools/conv_bench.py --batch $B --split --only expand --md $O/sweep_fp32_b$B.md > $O/sweep$B.log 2>&1 || { tail -20 $O/sweep$B.log; exit 1; }
cut -c1-150 $O/sweep$B.log
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/fp32.json 2> $O/fp32.err || { tail -20 $O/fp32.err; exit 1; }
python -c "import json;d=json.load(open('$O/fp32.json'));print('fp32',round(d['value']),d['p50_ms'],d['p99_ms'],d.get('avg_batch'),d.get('device_ms_per_batch'),round(d.get('direct_worker',{}).get('rps_this_rank',0)))"
