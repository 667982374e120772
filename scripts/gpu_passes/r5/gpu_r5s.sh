#!/usr/bin/env bash
# Round-5 pass S (item 3): the 4-rank rehearsal, count and process modes, with the harness's new
# default of 2 hardware queues per rank when ranks share one GPU.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 1
O=gpurun_out/${R5S_OUT:-r5s}; mkdir -p $O; export TMPDIR=/tmp PYTHONFAULTHANDLER=1
st() { echo "[r5s] $(date +%T) $*"; }
T="python bench/deploy_topology.py --ranks 4 --rehearsal --seconds 20 --producers 3 --rate 600000 --fmt json --trace"
for m in count process; do
  st $m
  X=""; [ $m = process ] && X="--standard-mode process --kie-shards 4"
  timeout -k 10 300 $T $X --log-dir $O/t4$m --out $O/topo4_$m.json > $O/topo4_$m.log 2>&1; rc=$?
  st "$m rc=$rc"; [ $rc -ge 2 ] && { tail -30 $O/topo4_$m.log; exit $rc; }
  python - $O/topo4_$m.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print({k: d.get(k) for k in ("value", "min_sample_tx_s", "incoming_equals_produced", "kie_standard_plus_fraud_equals_incoming",
                             "kie_duplicates", "arrival_to_scored_p50_us", "arrival_to_scored_p99_us", "checks_passed")})
print("produce->scored rows per rank", [r.get("rows") for r in d.get("produce_to_scored_us", [])])
for t in d.get("tail_attribution") or []:
    print(t["trace"][-9:], t["arrival_to_landed_us"], t["queued_us"], t.get("device_exec_us"), t.get("device_start_wait_us"),
          t.get("host_notice_us"), t.get("device_stall_windows"))
PY
done
st done
