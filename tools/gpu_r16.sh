set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=$GRAFT_REPO_ROOT/gpurun_out/r16
mkdir -p $O
timeout -k 10 600 python -m pytest tests/ -q -m gpu -s > $O/gpu_all.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && \
DIE_ROCTX=1 timeout -k 10 300 rocprofv3 --marker-trace --kernel-trace --stats --output-format csv -d $O/roctx -o m -- python3 bench.py --steps 30 --warmup 3 > $O/roctx.log 2>&1
echo "exit=$?"
