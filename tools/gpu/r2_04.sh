#!/bin/bash
# gateway forwarding loops sweep (fp32 + bf16), then a rocprofv3 kernel-stats pass of the fp32 headline
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2_04
mkdir -p $O
export DIE_TUNE_CACHE=$O/tune.json
summ() { python -c "import json;d=json.load(open('$1'));print('$2',round(d['value']),d['dtype'],d['config']['requests'],'p50',round(d['p50_ms'],2),'p99',round(d['p99_ms'],2),'avgB',round(d['avg_batch'],1),d.get('stages_us'),'direct',round(d.get('direct_worker',{}).get('rps_this_rank',0)))"; }
for t in 2 8 16; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --gw-client-threads $t > $O/fp32_t$t.json 2> $O/fp32_t$t.err || { tail -20 $O/fp32_t$t.err; exit 1; }
  summ $O/fp32_t$t.json fp32_t$t
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --precision bf16 > $O/bf16_auto.json 2> $O/bf16_auto.err || exit 1
summ $O/bf16_auto.json bf16_auto
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 2 --no-direct > $O/prof.json 2> $O/prof.err || { tail -20 $O/prof.err; exit 1; }
find $O/prof -name '*stats*' | head
