# round-6 stream-K probe: tests (unless $1 = notests), then cold sweeps of the stage-3/4 shapes with
# stream-K candidates
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r6sk2; mkdir -p $O
if [ "$1" != notests ]; then
timeout -k 10 500 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_splitk.py tests/test_gpu_ln_stats.py tests/test_gpu_general.py -k "streamk or fused_splitk or tail or stats" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python3 -u -m pytest -x -q -s --timeout 120 --timeout-method thread -m gpu tests/test_gpu_general.py -k offset > $O/offsets.log 2>&1 || { tail -20 $O/offsets.log; exit 1; }
grep -h "rel-L2" $O/offsets.log
fi
for s in s3.reduce s4.reduce s4.expand s3.expand s3.u0.proj s4.u0.proj s3.3x3 s4.3x3; do
timeout -k 10 200 python3 tools/conv_bench.py --batch 24 --split --cold --dump --trials 5 --only $s --cfgs 4,5,6,7,20,21,22,23,27 --splits 1,2,4 --sk 256,512,1024 > $O/cold_$s.txt 2>&1 || exit 1
done
