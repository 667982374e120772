#!/bin/bash
# Round 4: the deployed topology after the broker long poll and write-behind, and the native
# consumer's parallel JSON parse: GPU tests that drive kafka-lite; TXB1 durable vs in-memory
# broker; JSON 1.2e6/s with 1 / 2 / 4 parse threads; process mode; a kafka-lite SIGKILL +
# restart mid-run (exactly once with write-behind).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4n
mkdir -p $O
step() { echo "[r4n] $(date +%T) $*"; }
step pytest engine service / serve
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread \
  -k "engine_service or serve or scored" > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
show() { python3 -c "
import json,sys; d=json.load(open(sys.argv[1]))
print(d['value'], d['min_sample_tx_s'], d['producers_tx_s'], 'a->s', d['arrival_to_scored_p50_us'], d['arrival_to_scored_p99_us'], 'checks', d['checks_passed'], d.get('kie_standard_plus_fraud_equals_incoming'), 'durable', d.get('kafka_durable'))
print('produce->scored', d['produce_to_scored_us'])
print('scored->started', d['scored_to_process_started_us'])
if d.get('kafka_outage'): print('outage', d['kafka_outage'], d['incoming_equals_produced'], d['kie_duplicates'])" "$1"; }
run() {
  local n=$1; shift
  step $n
  timeout -k 30 300 python bench/deploy_topology.py --seconds 30 "$@" --log-dir $O/$n --out $O/$n.json > $O/$n.log 2>&1 \
    || { tail -40 $O/$n.log; exit 1; }
  show $O/$n.json
}
run txb1_durable --producers 4 --rate 0 --fmt txb1
run txb1_memory --producers 4 --rate 0 --fmt txb1 --kafka-memory
run json_p1 --producers 3 --rate 1200000 --fmt json
CCFD_KC_PARSE_THREADS=2 run json_p2 --producers 3 --rate 1200000 --fmt json
CCFD_KC_PARSE_THREADS=4 run json_p4 --producers 3 --rate 1200000 --fmt json
run json_process --producers 2 --rate 200000 --fmt json --standard-mode process
run json_kafka_kill --producers 3 --rate 1200000 --fmt json --kafka-kill-at 12 --kafka-down-s 2
step done
