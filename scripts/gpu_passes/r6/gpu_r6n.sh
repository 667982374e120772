#!/usr/bin/env bash
# Round-6 pass N: a 10-minute RF-3 JSON soak on the final defaults (3 brokers, 3-member controller
# quorum, thread fetchers, 1024-message produces) at 1.2e6 tx/s: every 5 s sample, the tail over
# the whole window, broker CPU and memory at the end.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 1
O=gpurun_out/r6n; mkdir -p $O; export TMPDIR=/tmp PYTHONFAULTHANDLER=1
st() { echo "[r6n] $(date +%T) $*"; }
st soak
timeout -k 10 900 python -u bench/deploy_topology.py --kafka-replicated --kafka-controllers 3 --rate 1.2e6 --seconds 600 \
  --fmt json --log-dir $O/soak --out $O/rf3_json_soak600.json 2>&1 | tee $O/soak.log | grep --line-buffered "sample" | awk 'NR % 6 == 0 { print; fflush() }'
rc=${PIPESTATUS[0]}
[ $rc -eq 0 ] || { tail -30 $O/soak.log; exit 1; }
python3 - $O/rf3_json_soak600.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
p = d["produce_to_scored_us"][0]
s = [x["tx_s"] for x in d["samples"]]
print({k: d.get(k) for k in ("value", "min_sample_tx_s", "incoming_equals_produced", "kie_duplicates", "checks_passed",
                             "produced_total", "kafka_data_bytes")}, "p2s p50/p99", p["p50"], p["p99"],
      "samples", len(s), "cpu", {k: v for k, v in d["cpu_s_by_service"].items() if k.startswith("kafka")})
PY
rm -rf $O/soak/kafka-lite* 2>/dev/null
st done
