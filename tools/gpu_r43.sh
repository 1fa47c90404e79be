#!/bin/bash
# side-stream projection branches: numerics + A/B on the headline bench and engine-only forward
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r43
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit 1
tail -2 $O/tests.log
for B in 16 24 32; do
  timeout -k 10 200 python bench.py --mode engine --batch $B --steps 200 --warmup 10 > $O/e$B.json 2> $O/e$B.err || exit 1
  timeout -k 10 200 python bench.py --mode engine --batch $B --steps 200 --warmup 10 --no-branch-streams > $O/e${B}n.json 2> $O/e${B}n.err || exit 1
  python -c "import json;a=json.load(open('$O/e$B.json'));b=json.load(open('$O/e${B}n.json'));print('engine B=$B dev ms: branches',round(a['device_ms_per_batch'],4),'inline',round(b['device_ms_per_batch'],4))"
done
i=0
for cfg in "" "--no-branch-streams" "" "--no-branch-streams"; do
  i=$((i+1))
  timeout -k 10 200 python bench.py --steps 400 --warmup 20 $cfg > $O/b$i.json 2> $O/b$i.err || exit 1
  echo "b$i [$cfg] $(python -c "import json,sys;d=json.load(open('$O/b$i.json'));print(round(d['value']),d['p50_ms'],d['p99_ms'],round(d['avg_batch'],1),round(d['device_ms_per_batch'],3),d.get('pace_lead_ms'),d.get('branch_streams'))")"
done
