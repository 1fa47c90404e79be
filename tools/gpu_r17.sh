#!/bin/bash
# conv ring-depth variants: numerics + race screen, then the per-shape sweep at batch 16 and 32
set -o pipefail
mkdir -p gpurun_out/r17
timeout -k 10 400 python -m pytest tests/test_gpu_kernels.py -x -q -k "conv" > gpurun_out/r17/tests.log 2>&1 &&
timeout -k 10 300 python tools/conv_bench.py --batch 16 --json gpurun_out/r17/conv_b16.json --md gpurun_out/r17/conv_b16.md > gpurun_out/r17/b16.log 2>&1 &&
timeout -k 10 300 python tools/conv_bench.py --batch 32 --json gpurun_out/r17/conv_b32.json --md gpurun_out/r17/conv_b32.md > gpurun_out/r17/b32.log 2>&1
