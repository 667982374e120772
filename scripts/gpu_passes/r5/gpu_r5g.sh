#!/usr/bin/env bash
# Round-5 pass G (VERDICT r4 items 4 + 3): the replicated multi-process kafka-lite (a controller
# + 3 broker processes, acks=all, pipelined idempotent producers) in the deployed topology --
# JSON 60 s without and with a broker SIGKILL, TXB1 with 8 producers -- then the 4-rank
# rehearsal with the stage trace + tail attribution, count and process modes.
# A step whose checks fail (rc 1) does not stop the pass; a crash, abort or time limit does.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 1
O=gpurun_out/r5g; mkdir -p $O; export TMPDIR=/tmp PYTHONFAULTHANDLER=1
st() { echo "[r5g] $(date +%T) $*"; }
run() {   # run <name> <seconds> <cmd...>
  local n=$1 t=$2; shift 2
  st "$n"
  timeout -k 10 "$t" "$@" > $O/$n.log 2>&1; local rc=$?
  st "$n rc=$rc"
  if [ $rc -ne 0 ]; then grep "\[deploy\]" $O/$n.log | tail -8; tail -25 $O/$n.log; fi
  if [ $rc -ge 2 ]; then exit $rc; fi
  [ -f $O/$n.json ] && python - $O/$n.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
keys = ("value", "min_sample_tx_s", "min_sample_ratio", "incoming_equals_produced", "kie_duplicates",
        "under_replicated_max", "under_replicated_final", "kafka_outage", "produce_to_scored_us",
        "arrival_to_scored_p50_us", "arrival_to_scored_p99_us", "checks_passed")
print({k: d.get(k) for k in keys if k in d})
print("samples", [s.get("tx_s") for s in d.get("samples", [])])
print("selectors", d.get("reference_dashboards", {}).get("matched"), "/", d.get("reference_dashboards", {}).get("selectors"))
for t in d.get("tail_attribution") or []:
    print("tail", json.dumps(t)[:1500])
PY
  return 0
}
R="python bench/deploy_topology.py --kafka-replicated --producer-acks -1 --producer-max-in-flight 5"
run repl_json_60s 300 $R --seconds 60 --producers 3 --rate 1.2e6 --fmt json --log-dir $O/rj --out $O/repl_json_60s.json
run repl_json_60s_kill 330 $R --seconds 60 --producers 3 --rate 1.2e6 --fmt json --kafka-kill-at 25 --kafka-down-s 5 \
    --kafka-kill-node 2 --log-dir $O/rjk --out $O/repl_json_60s_kill.json
run repl_txb1_p8 240 $R --seconds 30 --producers 8 --rate 0 --fmt txb1 --log-dir $O/rt --out $O/repl_txb1_p8.json
T="python bench/deploy_topology.py --ranks 4 --rehearsal --seconds 20 --producers 3 --rate 600000 --fmt json --trace"
run topo4_count 300 $T --log-dir $O/t4c --out $O/topo4_count.json
run topo4_process 300 $T --standard-mode process --kie-shards 4 --log-dir $O/t4p --out $O/topo4_process.json
st done
