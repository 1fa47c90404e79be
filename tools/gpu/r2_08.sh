#!/bin/bash
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2_08
mkdir -p $O
export DIE_TUNE_CACHE=$O/tune.json
timeout -k 10 600 python -u -m pytest tests/test_gpu_op_coverage.py -x -v --timeout 300 --timeout-method thread > $O/cov.log 2>&1 || { tail -40 $O/cov.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" $O/cov.log | tail -12
timeout -k 10 600 python -u -m pytest tests/test_gpu_cluster.py -x -v -s --timeout 300 --timeout-method thread > $O/cluster.log 2>&1 || { grep -E "CONFIG3|Error|assert" $O/cluster.log | cut -c1-700; exit 1; }
grep -E "CONFIG3|passed|failed" $O/cluster.log | cut -c1-700
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
