#!/bin/bash
# state check: GPU suite, smoke, headline x3, engine forwards, ViT headline
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r54
mkdir -p $O
export DIE_TUNE_CACHE=$O/tune.json
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit 1
tail -1 $O/tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
tail -1 $O/smoke.log
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 1500 --warmup 30 > $O/b$i.json 2> $O/b$i.err || exit 1
  echo "b$i $(python -c "import json,sys;d=json.load(open('$O/b$i.json'));print(round(d['value']),d['p50_ms'],d['p99_ms'],round(d['avg_batch'],1),round(d['device_ms_per_batch'],3),round(d.get('pace_lead_ms'),3))")"
done
for B in 16 24 32; do
  timeout -k 10 300 python bench.py --mode engine --batch $B --steps 300 --warmup 10 > $O/e$B.json 2> $O/e$B.err || exit 1
  python -c "import json;a=json.load(open('$O/e$B.json'));print('engine B=$B dev ms',round(a['device_ms_per_batch'],4))"
done
timeout -k 10 300 python bench.py --arch vit_b16 --steps 1000 --warmup 20 > $O/vit.json 2> $O/vit.err || exit 1
python -c "import json,sys;d=json.load(open('$O/vit.json'));print('vit',round(d['value']),d['p50_ms'],d['p99_ms'],round(d['avg_batch'],1),round(d['device_ms_per_batch'],3))"
timeout -k 10 300 python bench.py --mode dp --steps 600 --warmup 20 > $O/dp.json 2> $O/dp.err || exit 1
python -c "import json,sys;d=json.load(open('$O/dp.json'));print('dp1',round(d['value']),d['p50_ms'],d['p99_ms'],round(d['avg_batch'],1))"
