#!/usr/bin/env bash
# Live-cluster smoke check (reference diagnostics.sh behaviour, reimplemented): processes, ports,
# worker /health, gateway /stats, a direct worker /infer and a gateway /infer.
#   tools/diagnostics.sh [gateway_port=8000] [worker_ports="8001 8002 8003"]
GW_PORT=${1:-8000}
WORKER_PORTS=${2:-"8001 8002 8003"}
PAYLOAD='{"request_id":"diag_1","input_data":[1.0,2.0,3.0,4.0]}'
ok=0; bad=0
pass() { echo "  [ok]   $*"; ok=$((ok+1)); }
fail() { echo "  [FAIL] $*"; bad=$((bad+1)); }

echo "== processes"
for p in worker_node gateway; do
  n=$(ps -eo comm= | grep -cx "$p")
  [ "$n" -gt 0 ] && pass "$p running ($n)" || fail "$p not running"
done

echo "== ports"
for port in $GW_PORT $WORKER_PORTS; do
  if (exec 3<>/dev/tcp/127.0.0.1/$port) 2>/dev/null; then pass "port $port open"; else fail "port $port closed"; fi
done

echo "== worker health"
for port in $WORKER_PORTS; do
  h=$(curl -s -m 5 "http://127.0.0.1:$port/health")
  if echo "$h" | python3 -c 'import json,sys; d=json.load(sys.stdin); assert d["healthy"]; print("    node=%s requests=%s cache_hits=%s batches=%s engine=%s" % (d["node_id"], d["total_requests"], d["cache_hits"], d["batch_processor"]["total_batches"], d.get("engine",{}).get("name")))' 2>/dev/null; then
    pass "worker :$port healthy"
  else fail "worker :$port /health"; fi
done

echo "== gateway stats"
s=$(curl -s -m 5 "http://127.0.0.1:$GW_PORT/stats")
if echo "$s" | python3 -c 'import json,sys; d=json.load(sys.stdin); print("    workers=%d" % d["total_workers"]); [print("    %s %s failures=%d" % (b["node"], b["state"], b["failures"])) for b in d["circuit_breakers"]]' 2>/dev/null; then
  pass "gateway /stats"
else fail "gateway /stats"; fi

echo "== direct worker /infer"
first=$(echo $WORKER_PORTS | awk '{print $1}')
r=$(curl -s -m 30 -X POST -H 'Content-Type: application/json' -d "$PAYLOAD" "http://127.0.0.1:$first/infer")
echo "$r" | grep -q '"output_data"' && pass "worker :$first /infer" || fail "worker :$first /infer: $r"

echo "== gateway /infer"
r=$(curl -s -m 30 -X POST -H 'Content-Type: application/json' -d "$PAYLOAD" "http://127.0.0.1:$GW_PORT/infer")
echo "$r" | grep -q '"output_data"' && pass "gateway /infer" || fail "gateway /infer: $r"

echo "== $ok passed, $bad failed"
[ "$bad" -eq 0 ]
