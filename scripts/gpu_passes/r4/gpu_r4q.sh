#!/bin/bash
# Round 4, the committed tree: config 5 sustained for 60 s (JSON, durable broker), the same
# with a kafka-lite SIGKILL + restart at 25 s, and 4 engine ranks on one GPU (gloo rehearsal).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4q
mkdir -p $O
step() { echo "[r4q] $(date +%T) $*"; }
show() { python3 -c "
import json,sys; d=json.load(open(sys.argv[1]))
print(d['value'], d['min_sample_tx_s'], 'checks', d['checks_passed'], 'in==prod', d['incoming_equals_produced'], 'dups', d['kie_duplicates'], 'a->s', d['arrival_to_scored_p50_us'], d['arrival_to_scored_p99_us'])
print('samples', [s['tx_s'] for s in d['samples']])
print('produce->scored', d['produce_to_scored_us'])
print('scored->started', d['scored_to_process_started_us'])
if d.get('kafka_outage'): print('outage', d['kafka_outage'])
print('dashboards', d['reference_dashboards']['matched'], '/', d['reference_dashboards']['selectors'])" "$1"; }
run() {
  local n=$1; shift
  step $n
  timeout -k 30 400 python bench/deploy_topology.py "$@" --log-dir $O/$n --out $O/$n.json > $O/$n.log 2>&1 \
    || { tail -40 $O/$n.log; exit 1; }
  show $O/$n.json
}
run json60 --seconds 60 --producers 3 --rate 1200000 --fmt json
run json60_kafka_kill --seconds 60 --producers 3 --rate 1200000 --fmt json --kafka-kill-at 25 --kafka-down-s 2
run topo4_rehearsal --ranks 4 --rehearsal --seconds 20 --producers 3 --rate 600000 --fmt json --standard-mode process
step done
