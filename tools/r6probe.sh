# round-6: DMA-only / MFMA-only probes of the 3x3 kernels at B=24 (cold and warm)
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r6probe; mkdir -p $O
for pr in 0 1 2; do for mode in --cold ""; do
timeout -k 10 200 python3 tools/conv_bench.py --batch 24 --split $mode --dump --trials 5 --only s3.3x3 --cfgs 27,39,23 --splits 1,2 --probe $pr > $O/s3_p${pr}${mode}.txt 2>&1 || exit 1
done; done
