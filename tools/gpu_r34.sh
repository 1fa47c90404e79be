#!/bin/bash
# conv loop without divisions/selects: numerics, race screen, sweep at batch 16/32
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r34
mkdir -p $O
timeout -k 10 900 python -m pytest tests/ -m gpu -x -q > $O/tests.log 2>&1 || exit 1
timeout -k 10 300 python tools/conv_bench.py --batch 16 --json $O/conv_b16.json --md $O/conv_b16.md > $O/b16.log 2>&1 || exit 1
timeout -k 10 300 python tools/conv_bench.py --batch 32 --json $O/conv_b32.json --md $O/conv_b32.md > $O/b32.log 2>&1 || exit 1
timeout -k 10 240 python bench.py --steps 300 --warmup 10 > $O/bench.json 2> $O/bench.err || exit 1
echo done
