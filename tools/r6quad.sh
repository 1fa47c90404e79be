# round-6 four-tile 3x3 kernel (variant 9): tests, cold sweep of the 3x3 shapes, then (ops) a B=24 op profile
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r6quad3; mkdir -p $O
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_splitk.py -k quad > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for s in s3.3x3 s4.3x3 s2.3x3; do
timeout -k 10 200 python3 tools/conv_bench.py --batch 24 --split --cold --dump --trials 5 --only $s --cfgs 27,39 --splits 1,2,4,8 > $O/cold_$s.txt 2>&1 || exit 1
done
if [ "$1" = ops ]; then bash tools/gpu_run.sh r6quad3 ops resnet50 24 fp32 || exit 1; fi
exit 0
