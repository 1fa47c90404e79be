#!/bin/bash
# Final-state evidence: per-op fp32 profiles at the serving batch (20) and at 32, rocprofv3 kernel
# stats of the headline bench.
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2_31
mkdir -p $O
export DIE_TUNE_CACHE=$O/tune.json
cd /tmp && export TMPDIR=/tmp
cd $R
for B in 20 32; do
  timeout -k 10 300 python -u tools/op_profile.py --arch resnet50 --batch $B --precision fp32 --out $O/ops_fp32_b$B.md > $O/ops_$B.log 2>&1 || { tail -20 $O/ops_$B.log; exit 1; }
  sed -n 3p $O/ops_fp32_b$B.md.md
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o bench -- python3 bench.py --steps 20 --warmup 5 > $O/bench_prof.json 2> $O/bench_prof.err || { tail -20 $O/bench_prof.err; exit 1; }
cut -c1-300 $O/bench_prof.json
find $O/prof -name "*kernel_stats*" | head -3
