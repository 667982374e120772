#!/usr/bin/env bash
# Round-5 pass B: config 5 with the reference's semantics (a process for EVERY transaction) on a
# sharded KIE tier: a 20 s shake-down, then 60 s at 1.2e6 JSON tx/s with KIE
# shard 1 SIGKILLed at 25 s and restarted from its journal 5 s later.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 1
O=gpurun_out/r5b; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python bench/deploy_topology.py --standard-mode process --kie-shards 4 --rate 1.2e6 \
    --seconds 20 --producers 3 --fmt json --log-dir $O/shake --out $O/process_k4_20s.json > $O/shake.log 2>&1 \
    || { tail -c 3000 $O/shake.log; for f in $O/shake/*.log; do echo "== $f"; tail -15 $f; done; exit 1; }
python -c "import json; d=json.load(open('$O/process_k4_20s.json')); print({k: d.get(k) for k in ('value','min_sample_tx_s','incoming_equals_produced','kie_standard_plus_fraud_equals_incoming','kie_duplicates','kie_standard_duplicates','scored_to_process_started_us','checks_passed')})"
timeout -k 10 500 python bench/deploy_topology.py --standard-mode process --kie-shards 4 --rate 1.2e6 \
    --seconds 60 --producers 3 --fmt json --kie-outage-at 25 --kie-kill-shard 1 --kie-outage-s 5 \
    --log-dir $O/kill --out $O/process_k4_60s_kill.json > $O/kill.log 2>&1 \
    || { tail -c 3000 $O/kill.log; for f in $O/kill/*.log; do echo "== $f"; tail -15 $f; done; exit 1; }
python -c "import json; d=json.load(open('$O/process_k4_60s_kill.json')); print({k: d.get(k) for k in ('value','min_sample_tx_s','incoming_equals_produced','kie_standard_plus_fraud_equals_incoming','kie_duplicates','kie_standard_duplicates','scored_to_process_started_us','kie_outage','checks_passed')})"
