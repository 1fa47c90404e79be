# round-6: GPU tests (files given after the output name) and the B=24 ResNet50 per-op profile
# usage: bash tools/r6run.sh <out-name> [test files...]
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/$1; shift; mkdir -p $O
if [ $# -gt 0 ]; then
  timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread "$@" > $O/tests.txt 2>&1 || exit 1
fi
timeout -k 10 400 python3 tools/op_profile.py --arch resnet50 --batch 24 --out $O/ops_b24 > $O/ops.txt 2>&1 || exit 1
