#!/usr/bin/env bash
# Round-6 pass L: the fail-over drills again on the new kafka-lite defaults (follower fetch on a
# thread per leader, 1024-message JSON produces): a broker SIGKILL (the node leading partitions
# and replicating the others) and an active-controller SIGKILL, RF-3 JSON at 1.2e6 tx/s.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 1
O=gpurun_out/r6l; mkdir -p $O; export TMPDIR=/tmp PYTHONFAULTHANDLER=1
st() { echo "[r6l] $(date +%T) $*"; }
summ() {
python3 - $1 <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
p = d["produce_to_scored_us"][0]
print({k: d.get(k) for k in ("value", "min_sample_tx_s", "incoming_equals_produced", "kie_duplicates", "checks_passed",
                             "producer_batch")}, "p2s p50/p99", p["p50"], p["p99"],
      {k: v for k, v in d.items() if "controller" in k and not isinstance(v, (dict, list))})
PY
}
st broker kill
timeout -k 10 330 python -u bench/deploy_topology.py --kafka-replicated --kafka-controllers 3 --rate 1.2e6 --seconds 60 \
  --fmt json --kafka-kill-at 25 --kafka-down-s 5 --kafka-kill-node 2 --log-dir $O/bk --out $O/rf3_json_broker_kill.json \
  > $O/broker_kill.log 2>&1 || { tail -30 $O/broker_kill.log; exit 1; }
summ $O/rf3_json_broker_kill.json
st controller kill
timeout -k 10 330 python -u bench/deploy_topology.py --kafka-replicated --kafka-controllers 3 --rate 1.2e6 --seconds 60 \
  --fmt json --controller-kill-at 25 --controller-down-s 5 --log-dir $O/ck --out $O/rf3_json_controller_kill.json \
  > $O/controller_kill.log 2>&1 || { tail -30 $O/controller_kill.log; exit 1; }
summ $O/rf3_json_controller_kill.json
rm -rf $O/bk/kafka-lite* $O/ck/kafka-lite* 2>/dev/null
st done
