#!/bin/bash
# fp32 (split) kernels: numerics tests first, then the whole GPU suite
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2_02
mkdir -p $O
export DIE_TUNE_CACHE=$O/tune.json
timeout -k 10 900 python -u -m pytest tests/test_gpu_fp32.py -x -v -s --timeout 300 --timeout-method thread > $O/fp32.log 2>&1 || { tail -40 $O/fp32.log; exit 1; }
grep -E "passed|failed|rel-L2" $O/fp32.log | tail -12
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
