#!/bin/bash
# Multi-rank rehearsal of the driver's N-GPU launch on the 1-GPU box: torchrun, 2 ranks sharing
# GPU 0, gateway mode (each rank's gateway routes over both ranks' workers; cross-process
# shared-memory bodies), exactly the driver's command line at N=2.
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2_52
mkdir -p $O
export DIE_TUNE_CACHE=$O/tune.json
cd $R
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 20 --warmup 4 > $O/n2.json 2> $O/n2.err || { tail -30 $O/n2.err; exit 1; }
cat $O/n2.json | cut -c1-1500
