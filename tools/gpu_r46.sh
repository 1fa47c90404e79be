#!/bin/bash
# cold-L2 autotune vs warm back-to-back autotune: engine forward + headline
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r46
mkdir -p $O
export DIE_TUNE_CACHE=$O/tune.json
for B in 16 24 32; do
  for w in 0 1; do
    s=$(date +%s.%N)
    DIE_TUNE_WARM=$w timeout -k 10 300 python bench.py --mode engine --batch $B --steps 200 --warmup 10 > $O/e${B}_$w.json 2> $O/e${B}_$w.err || exit 1
    e=$(date +%s.%N)
    python -c "import json;a=json.load(open('$O/e${B}_$w.json'));print('engine B=$B warm=$w dev ms',round(a['device_ms_per_batch'],4),'wall s', round($e-$s,1))"
  done
done
i=0
for w in 0 1 0 1; do
  i=$((i+1))
  DIE_TUNE_WARM=$w timeout -k 10 300 python bench.py --steps 400 --warmup 20 > $O/b$i.json 2> $O/b$i.err || exit 1
  echo "b$i [warm=$w] $(python -c "import json,sys;d=json.load(open('$O/b$i.json'));print(round(d['value']),d['p50_ms'],d['p99_ms'],round(d['avg_batch'],1),round(d['device_ms_per_batch'],3),round(d.get('pace_lead_ms'),3),d['worker_init_s'])")"
done
