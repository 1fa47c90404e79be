# Same-box A/B of bench.py: the baseline library build (ab/libdie_base.so via DIE_LIB_PATH) against
# the in-tree one, interleaved.  usage: bash tools/ab_bench.sh <out-name> <rounds> [bench.py args]
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
export DIE_TUNE_CACHE=${DIE_TUNE_CACHE:-$PWD/tools/tune_r6_final.json}
O=gpurun_out/$1; R=$2; shift 2; mkdir -p $O
for r in $(seq 1 $R); do
  DIE_LIB_PATH=$PWD/ab/libdie_base.so timeout -k 10 300 python3 bench.py "$@" > $O/base_$r.json 2> $O/base_$r.err || exit 1
  timeout -k 10 300 python3 bench.py "$@" > $O/new_$r.json 2> $O/new_$r.err || exit 1
  for a in base new; do
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); g=d.get('gateway_bytes') or {}; w=d.get('direct_worker') or {}; print(sys.argv[2], round(d['value']), d['avg_batch'], 'bytes', round(g.get('requests_per_s',0)), g.get('p50_ms'), 'direct', round(w.get('rps_this_rank',0)), 'cpu', d.get('cpu_us_per_request'))" $O/${a}_$r.json ${a}_$r
  done
done
