# round-6: DP leader merge target balanced (default) vs not, world 1 with the merge path forced,
# interleaved rounds on one box.  usage: bash tools/r6dp.sh <out-name> [rounds]
# (the --no-dp-balance flag and EngineOptions::dp_balance were removed with the revert: profiles/r6_dp_balance_ab.md)
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
export DIE_TUNE_CACHE=${DIE_TUNE_CACHE:-$PWD/tools/tune_r6_final.json}
O=gpurun_out/$1; R=${2:-3}; mkdir -p $O
for r in $(seq 1 $R); do
  for v in bal nobal; do
    extra=""; [ $v = nobal ] && extra="--no-dp-balance"
    MASTER_ADDR=127.0.0.1 MASTER_PORT=$((29500 + r)) RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 \
      timeout -k 10 240 python3 bench.py --mode dp --gpus 1 --dp-force-merge --steps 20 --warmup 5 $extra \
      > $O/${v}_$r.json 2> $O/${v}_$r.err || exit 1
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['value']), d.get('p50_ms'), d.get('p99_ms'), d.get('avg_dp_batch'))" $O/${v}_$r.json ${v}_$r
  done
done
