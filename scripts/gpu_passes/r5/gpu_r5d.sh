#!/usr/bin/env bash
# Round-5 pass D: the hand-off back-pressure path under process mode (new GPU test), then pass
# B's 60 s KIE-shard kill again with faulthandler on every service.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 1
O=gpurun_out/r5d; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_engine_service_gpu.py -x -v --timeout 200 --timeout-method thread \
    -k "back_pressure or standard_mode_process" > $O/pytest.log 2>&1 || { tail -80 $O/pytest.log; exit 1; }
tail -4 $O/pytest.log
timeout -k 10 500 python bench/deploy_topology.py --standard-mode process --kie-shards 4 --rate 1.2e6 \
    --seconds 60 --producers 3 --fmt json --kie-outage-at 25 --kie-kill-shard 1 --kie-outage-s 5 \
    --log-dir $O/kill --out $O/process_k4_60s_kill.json > $O/kill.log 2>&1 \
    || { grep "\[deploy\]" $O/kill.log | tail -20; for f in $O/kill/engine.log $O/kill/kie1-restarted.log; do echo "== $f"; tail -80 $f; done; exit 1; }
python -c "import json; d=json.load(open('$O/process_k4_60s_kill.json')); print({k: d.get(k) for k in ('value','min_sample_tx_s','samples','incoming_equals_produced','kie_standard_plus_fraud_equals_incoming','kie_duplicates','kie_standard_duplicates','scored_to_process_started_us','kie_outage','checks_passed')})"
