#!/usr/bin/env bash
# Round-5 pass C: the KIE-shard kill under process mode again, with faulthandler on (pass B's
# engine died with SIGSEGV after the killed shard came back).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 1
O=gpurun_out/r5c; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python bench/deploy_topology.py --standard-mode process --kie-shards 4 --rate 1.2e6 \
    --seconds 40 --producers 3 --fmt json --kie-outage-at 15 --kie-kill-shard 1 --kie-outage-s 5 \
    --log-dir $O/kill --out $O/process_k4_40s_kill.json > $O/kill.log 2>&1 \
    || { grep "\[deploy\]" $O/kill.log | tail -20; for f in $O/kill/*.log; do echo "== $f"; tail -60 $f; done; exit 1; }
python -c "import json; d=json.load(open('$O/process_k4_40s_kill.json')); print({k: d.get(k) for k in ('value','min_sample_tx_s','samples','incoming_equals_produced','kie_standard_plus_fraud_equals_incoming','kie_duplicates','kie_standard_duplicates','scored_to_process_started_us','kie_outage','checks_passed')})"
