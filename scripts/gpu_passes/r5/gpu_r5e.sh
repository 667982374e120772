#!/usr/bin/env bash
# Round-5 pass E (VERDICT r4 items 1 + 2): the hand-off back-pressure GPU test after the
# engine-destroy fix; config 5 in process mode on 4 KIE shards for 60 s without and with a KIE
# shard SIGKILL; the notification loop over the same transactions without and with KIE + notifier
# SIGKILLs (outcomes compared process for process through the outcome digest).
# A step whose checks fail (rc 1) does not stop the pass; a crash, abort or time limit does.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 1
O=gpurun_out/r5e; mkdir -p $O; export TMPDIR=/tmp PYTHONFAULTHANDLER=1
st() { echo "[r5e] $(date +%T) $*"; }
run() {   # run <name> <seconds> <cmd...>: output in $O/<name>.log
  local n=$1 t=$2; shift 2
  st "$n"
  timeout -k 10 "$t" "$@" > $O/$n.log 2>&1; local rc=$?
  st "$n rc=$rc"
  if [ $rc -ne 0 ]; then grep "\[deploy\]" $O/$n.log | tail -8; tail -25 $O/$n.log; fi
  if [ $rc -ge 2 ]; then exit $rc; fi       # crash / abort / time limit: nothing more on the GPU
  return 0
}
summ() { python - "$@" <<'EOF'
import json, sys
d = json.load(open(sys.argv[1]))
keys = ("value", "min_sample_tx_s", "incoming_equals_produced", "kie_standard_plus_fraud_equals_incoming",
        "kie_duplicates", "kie_standard_duplicates", "scored_to_process_started_us", "kie_outage", "notifier_outage",
        "kie_notified_equals_fraud_started", "settled", "customer_replies_applied", "same_outcomes_as", "checks_passed")
print({k: d.get(k) for k in keys if k in d})
print("outcomes", d.get("kie", {}).get("outcomes"), d.get("kie", {}).get("outcome_digest"),
      "selectors", d.get("reference_dashboards", {}).get("matched"), "/", d.get("reference_dashboards", {}).get("selectors"))
EOF
}
run bp_pytest 280 python -u -m pytest tests/test_engine_service_gpu.py -x -v --timeout 200 --timeout-method thread -k back_pressure
tail -3 $O/bp_pytest.log
P="python bench/deploy_topology.py --standard-mode process --kie-shards 4 --rate 1.2e6 --producers 3 --fmt json"
run process_60s 330 $P --seconds 60 --log-dir $O/p60 --out $O/process_k4_60s.json
[ -f $O/process_k4_60s.json ] && summ $O/process_k4_60s.json
run process_60s_kill 360 $P --seconds 60 --kie-outage-at 25 --kie-kill-shard 1 --kie-outage-s 5 \
    --log-dir $O/p60k --out $O/process_k4_60s_kill.json
[ -f $O/process_k4_60s_kill.json ] && summ $O/process_k4_60s_kill.json
N="python bench/deploy_topology.py --kie-shards 2 --rate 1.0e6 --producers 2 --fmt json --count 10000000 --seconds 30 \
   --settle --notification-timeout-s 20 --notifier-seed 7"
run notif_ref 300 $N --log-dir $O/nref --out $O/notif_ref.json
[ -f $O/notif_ref.json ] && summ $O/notif_ref.json
run notif_crash 330 $N --kie-outage-at 8 --kie-kill-shard 0 --kie-outage-s 3 --notifier-kill-at 11 --notifier-down-s 3 \
    --compare-to $O/notif_ref.json --log-dir $O/ncrash --out $O/notif_crash.json
[ -f $O/notif_crash.json ] && summ $O/notif_crash.json
st done
