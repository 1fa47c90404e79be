set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r4
mkdir -p $O
timeout -k 10 600 python -m pytest tests/test_gpu_transformer.py -x -q > $O/tf.log 2>&1 && \
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py tests/test_gpu_engine.py -x -q > $O/kern.log 2>&1 && \
timeout -k 10 200 python tools/parse_bench.py > $O/parse.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 150 --warmup 5 > $O/bench.log 2>&1 && \
timeout -k 10 300 python bench.py --mode engine --arch vit_b16 --steps 50 --warmup 3 > $O/bench_vit_engine.log 2>&1 && \
timeout -k 10 300 python bench.py --arch vit_b16 --steps 60 --warmup 3 > $O/bench_vit.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o prof --output-format csv -- python bench.py --mode engine --arch vit_b16 --steps 10 --warmup 2 > $O/prof.log 2>&1
echo "exit=$?"
