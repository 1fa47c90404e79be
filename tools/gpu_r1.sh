set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py -x -q > gpurun_out/r1_kern.log 2>&1 && \
timeout -k 10 400 python -m pytest tests/test_gpu_engine.py -x -q > gpurun_out/r1_eng.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 40 --warmup 3 > gpurun_out/r1_bench.log 2>&1 && \
timeout -k 10 300 python bench.py --mode engine --steps 50 --warmup 5 > gpurun_out/r1_bench_engine.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r1_prof -o prof --output-format csv -- python bench.py --mode engine --steps 20 --warmup 2 > gpurun_out/r1_prof.log 2>&1
echo "exit=$?"
