#!/bin/bash
# re-entry check: GPU suite, smoke, headline bench (http) and engine-only forward
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r35
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 240 python bench.py --steps 300 --warmup 10 > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 240 python bench.py --mode engine --steps 200 --warmup 10 > $O/bench_engine.json 2> $O/bench_engine.err || exit 1
echo done
