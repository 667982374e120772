#!/usr/bin/env bash
# Round-6 pass B: deployed-topology drills.
#  1. reference semantics (a process per transaction, 4 KIE shards, ~1e6 JSON tx/s): KIE shard 1
#     SIGKILLed for 12 s and, 5 s into that outage, the engine crashed and restarted from its
#     committed offsets -- standard + fraud processes must equal the transactions produced;
#  2. RF-3 replicated kafka-lite with the 3-member controller quorum at 1.2e6 JSON tx/s, the
#     ACTIVE controller SIGKILLed at 25 s (restarted 5 s later).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 1
O=gpurun_out/r6b; mkdir -p $O; export TMPDIR=/tmp PYTHONFAULTHANDLER=1
st() { echo "[r6b] $(date +%T) $*"; }
st drill1
timeout -k 10 420 python -u bench/deploy_topology.py --standard-mode process --kie-shards 4 --rate 1.0e6 \
  --seconds 60 --fmt json --kie-outage-at 15 --kie-outage-s 12 --kie-kill-shard 1 --engine-kill-at 20 \
  --engine-down-s 3 --log-dir $O/drill1 --out $O/drill1.json > $O/drill1.log 2>&1
rc=$?
python - $O/drill1.json <<'PY' || true
import json, sys
d = json.load(open(sys.argv[1]))
keys = ["value", "min_sample_tx_s", "produced_total", "transaction_incoming_total", "kie_standard_plus_fraud_equals_produced",
        "kie_standard_duplicates", "kie_duplicates", "duplicates_recognised", "engine_outage", "kie_outage", "checks_passed"]
print({k: d.get(k) for k in keys})
PY
[ $rc -eq 0 ] || { st "drill1 rc=$rc"; tail -30 $O/drill1.log; exit 1; }
st drill2
timeout -k 10 420 python -u bench/deploy_topology.py --kafka-replicated --kafka-controllers 3 --rate 1.2e6 \
  --seconds 60 --fmt json --controller-kill-at 25 --controller-down-s 5 --log-dir $O/drill2 \
  --out $O/drill2.json > $O/drill2.log 2>&1
rc=$?
python - $O/drill2.json <<'PY' || true
import json, sys
d = json.load(open(sys.argv[1]))
keys = ["value", "min_sample_tx_s", "min_sample_ratio", "incoming_equals_produced", "kie_duplicates", "controller_outage",
        "produce_to_scored_us", "checks_passed"]
print({k: d.get(k) for k in keys})
print([s["tx_s"] for s in d["samples"]])
PY
[ $rc -eq 0 ] || { st "drill2 rc=$rc"; tail -30 $O/drill2.log; exit 1; }
st done
