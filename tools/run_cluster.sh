#!/usr/bin/env bash
# Start the README topology: 3 workers (one GPU each when available) + gateway on :8000.
#   tools/run_cluster.sh model.onnx [device=auto]      (Ctrl-C stops everything)
set -e
MODEL=${1:?usage: run_cluster.sh model.onnx [device]}
DEVICE=${2:-auto}
BIN="$(cd "$(dirname "$0")/.." && pwd)/distributed-inference-engine-cpp_amd/bin"
pids=()
trap 'kill "${pids[@]}" 2>/dev/null; wait' INT TERM EXIT
for i in 0 1 2; do
  "$BIN/worker_node" $((8001 + i)) "worker$((i + 1))" "$MODEL" --device "$DEVICE" --device-id $i &
  pids+=($!)
done
sleep 2
"$BIN/gateway" localhost:8001 localhost:8002 localhost:8003 --port 8000 &
pids+=($!)
wait
