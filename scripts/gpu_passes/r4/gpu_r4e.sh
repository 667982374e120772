#!/bin/bash
# Round 4: config 5 on the durable broker -- 60 s JSON at 1.2e6 tx/s without and with a
# kafka-lite SIGKILL + restart from disk at t = 25 s.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4e
mkdir -p $O
step() { echo "[r4e] $(date +%T) $*"; }
df -h /tmp . > $O/df.txt 2>&1; cat $O/df.txt
step json 60 s durable, no kill
timeout -k 30 420 python bench/deploy_topology.py --seconds 60 --producers 3 --rate 1200000 --fmt json \
  --log-dir $O/json60 --out $O/topo_json60_durable.json > $O/topo_json60_durable.log 2>&1 \
  || { tail -40 $O/topo_json60_durable.log; exit 1; }
python3 -c "import json; d=json.load(open('$O/topo_json60_durable.json')); print(d['value'], d['min_sample_tx_s'], d['checks_passed'], d['arrival_to_scored_p50_us'], d['arrival_to_scored_p99_us'], d.get('produce_to_scored_us'), d.get('scored_to_process_started_us'), d.get('kafka_data_bytes'))"
step json 60 s, kafka-lite SIGKILLed at 25 s
timeout -k 30 480 python bench/deploy_topology.py --seconds 60 --producers 3 --rate 1200000 --fmt json \
  --kafka-kill-at 25 --kafka-down-s 2 --log-dir $O/json60_kill --out $O/topo_json60_kafka_kill.json \
  > $O/topo_json60_kafka_kill.log 2>&1 || { tail -40 $O/topo_json60_kafka_kill.log; exit 1; }
python3 -c "import json; d=json.load(open('$O/topo_json60_kafka_kill.json')); print(d['value'], d['checks_passed'], d['incoming_equals_produced'], d['kie_duplicates'], d.get('kafka_outage'), [s['tx_s'] for s in d['samples']])"
step done
