# round-6: stem + pool kernel tests and the B=24 per-op profile
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/${1:-r6stem}; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_stem_pool.py \
  tests/test_gpu_fp32.py tests/test_gpu_gap_fc.py tests/test_gpu_kernels.py -k "stem or gap or pool" > $O/tests.txt 2>&1 || exit 1
timeout -k 10 400 python3 tools/op_profile.py --arch resnet50 --batch 24 --out $O/ops_b24 > $O/ops.txt 2>&1 || exit 1
