#!/bin/bash
# One parameterised runner for GPU-box work (replaces round 1-2's one-off tools/gpu_r*.sh scripts).
# Run on the box, e.g.  gpurun -- 'bash tools/gpu_run.sh <out-name> <task> [args...]'
#
# Every step runs under its own time limit and the chain stops at the first failure.  Results go to
# gpurun_out/<out-name>/ (merged back by gpurun); summaries worth keeping are copied to profiles/.
#
# tasks:
#   tests [pytest -k expr]        the GPU suite (-m gpu), one process, per-test timeouts
#   smoke                         __graft_entry__.smoke()
#   bench NAME [bench.py args]    one bench.py run -> NAME.json, one summary line
#   ab N NAME=ARGS...             N interleaved rounds of bench.py variants: "fp32=--precision fp32" ...
#   ops ARCH B PREC               per-op device time table (tools/op_profile.py)
#   rocprof NAME [bench.py args]  rocprofv3 --kernel-trace --stats around bench.py, summary via tools/prof_summary.py
#   pmc ARCH B PREC               4 PMC passes of one forward (tools/pmc_forward.py) -> pmc_<arch>_<prec>_b<B>.md
#   micro NAME                    a prebuilt tools/micro/NAME probe -> micro_NAME.md
#   refbench [ref_bench.py args]  the reference's benchmark.py run: gateway + 3 HIP workers on GPU 0 -> refbench.json
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
NAME=$1; TASK=$2; shift 2
O=$R/gpurun_out/$NAME
mkdir -p "$O"
export DIE_TUNE_CACHE=${DIE_TUNE_CACHE:-$O/tune.json}
cd "$R" || exit 1

summ() {  # one line per bench JSON
  python3 - "$1" "$2" <<'EOF'
import json, sys
d = json.load(open(sys.argv[1]))
dw = d.get("direct_worker", {})
dp = d.get("dp_rccl") or {}
print(sys.argv[2], round(d["value"]), "p50", d.get("p50_ms"), "p99", d.get("p99_ms"), "batch", d.get("avg_batch") or d.get("avg_dp_batch"),
      "dev_ms", d.get("device_ms_per_batch"), "gap_ms", d.get("gpu_gap_ms_per_batch"), "cache_hits", d.get("cache_hits_timed"),
      "trim", d.get("trimmed_batches"), "direct", round(dw.get("rps_this_rank", 0)), dw.get("p99_ms"), "dp_rccl", dp.get("requests_per_s"), dp.get("p99_ms"), dp.get("error", ""))
EOF
}

bench() {
  local n=$1; shift
  timeout -k 10 600 python3 bench.py "$@" > "$O/$n.json" 2> "$O/$n.err" || { tail -20 "$O/$n.err"; return 1; }
  summ "$O/$n.json" "$n"
}

case "$TASK" in
  tests)
    K=()
    [ -n "$1" ] && K=(-k "$1")
    timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread "${K[@]}" > "$O/tests.log" 2>&1 \
      || { grep -E "Error|assert|FAIL" "$O/tests.log" | cut -c1-300 | tail -20; tail -5 "$O/tests.log"; exit 1; }
    tail -2 "$O/tests.log" ;;
  smoke)
    timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { tail -20 "$O/smoke.log"; exit 1; }
    tail -1 "$O/smoke.log" ;;
  bench)
    n=$1; shift
    bench "$n" "$@" || exit 1 ;;
  ab)
    rounds=$1; shift
    for r in $(seq 1 "$rounds"); do
      for v in "$@"; do
        n=${v%%=*}; a=${v#*=}
        # shellcheck disable=SC2086
        bench "${n}_$r" $a || exit 1
      done
    done ;;
  abdir)  # abdir N NAME=DIR=ARGS...: as ab, each variant's bench.py run from its own tree DIR (same box)
    rounds=$1; shift
    for r in $(seq 1 "$rounds"); do
      for v in "$@"; do
        n=${v%%=*}; rest=${v#*=}; d=${rest%%=*}; a=${rest#*=}
        # shellcheck disable=SC2086
        (cd "$R/$d" && DIE_TUNE_CACHE=$O/tune_$n.json timeout -k 10 600 python3 bench.py $a > "$O/${n}_$r.json" 2> "$O/${n}_$r.err") \
          || { tail -20 "$O/${n}_$r.err"; exit 1; }
        summ "$O/${n}_$r.json" "${n}_$r"
      done
    done ;;
  ops)  # ops ARCH B PREC [TAG [op_profile.py args]]
    A=$1; B=$2; P=$3; T=${4:-}; shift 3; [ $# -gt 0 ] && shift
    timeout -k 10 300 python3 -u tools/op_profile.py --arch "$A" --batch "$B" --precision "$P" --out "$O/ops_${A}_${P}_b$B$T" "$@" \
      > "$O/ops$T.log" 2>&1 || { tail -20 "$O/ops$T.log"; exit 1; }
    sed -n 3p "$O/ops_${A}_${P}_b$B$T.md" ;;
  rocprof)
    n=$1; shift
    cd /tmp && export TMPDIR=/tmp && cd "$R" || exit 1
    timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/$n" -o p -- python3 bench.py --no-dp "$@" > "$O/$n.json" 2> "$O/$n.err" \
      || { tail -20 "$O/$n.err"; exit 1; }
    summ "$O/$n.json" "$n"
    # rocprofv3 (ROCm 7.2) writes a rocpd SQLite database by default, CSVs with --output-format csv
    f=$(find "$O/$n" -name '*_results.db' -print -quit)
    if [ -n "$f" ]; then
      python3 tools/rocpd_stats.py "$f" --top 40 --md "$O/$n.md" > /dev/null || exit 1
    else
      f=$(find "$O/$n" -name '*kernel_stats.csv' -print -quit)
      [ -n "$f" ] || { echo "no rocprofv3 output under $O/$n"; exit 1; }
      python3 tools/prof_summary.py "${f%_kernel_stats.csv}" > "$O/$n.md" || exit 1
    fi
    head -30 "$O/$n.md"
    rm -rf "${O:?}/$n" ;;
  pmc)
    A=$1; B=$2; P=$3; D=$O/pmc_${A}_${P}_b$B
    cd /tmp && export TMPDIR=/tmp && cd "$R" || exit 1
    run_pass() {
      local k=$1; shift
      timeout -s KILL 180 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d "$D/p$k" -o p -- \
        python3 tools/pmc_forward.py "$A" "$B" 2 "$P" tuned > "$D.p$k.log" 2>&1
    }
    run_pass 1 GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS && \
    run_pass 2 FETCH_SIZE && \
    run_pass 3 WRITE_SIZE TCC_HIT_sum TCC_MISS_sum && \
    run_pass 4 SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_MFMA \
      || { tail "$D".p*.log; exit 1; }
    python3 tools/pmc_summary.py "$D" --title "$A $P B=$B tuned" --note "production (autotuned) kernel configs, eager launches" \
      > "$O/pmc_${A}_${P}_b$B.md" || exit 1
    rm -rf "$D"  # raw traces: tens of MB, past gpurun's 64 MiB copy-back limit
    tail -1 "$O/pmc_${A}_${P}_b$B.md" ;;
  micro)  # a prebuilt tools/micro/<name> binary (built here: hipcc ... -o tools/micro/<name>)
    timeout -k 10 300 "tools/micro/$1" > "$O/micro_$1.md" 2>&1 || { tail -20 "$O/micro_$1.md"; exit 1; }
    cat "$O/micro_$1.md" ;;
  refbench)
    timeout -k 10 900 python3 -u tools/ref_bench.py --out "$O/refbench.json" --log-dir "$O/refbench_logs" "$@" \
      > "$O/refbench.log" 2>&1 || { tail -20 "$O/refbench.log"; exit 1; }
    tail -1 "$O/refbench.log" ;;
  *)
    echo "unknown task $TASK"; exit 2 ;;
esac
