#!/bin/bash
# decode fast path + GAP rework: GPU tests, decode bench, headline x2, engine B=20
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r56
mkdir -p $O
export DIE_TUNE_CACHE=$O/tune.json
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python tools/decode_bench.py > $O/decode.json 2> $O/decode.err || exit 1
cat $O/decode.json
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 1500 --warmup 30 > $O/b$i.json 2> $O/b$i.err || exit 1
  echo "b$i $(python -c "import json,sys;d=json.load(open('$O/b$i.json'));print(round(d['value']),d['p50_ms'],d['p99_ms'],round(d['avg_batch'],1),round(d['device_ms_per_batch'],3),d['prep_ms_per_batch'])")"
done
timeout -k 10 300 python tools/op_profile.py --arch resnet50 --batch 20 --out $O/ops_rn50_b20 > /dev/null 2>&1 || exit 1
grep -E "gap|dense|Total" $O/ops_rn50_b20.md | head -4
