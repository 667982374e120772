#!/usr/bin/env bash
# Round-6 pass E3: pass E again on the new defaults (follower fetch on a thread per leader,
# 1024-message JSON produce requests): five consecutive 60 s RF-3 JSON runs at 1.2e6 tx/s, produce -> scored
# p99 and the brokers CPU-seconds per run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 1
O=gpurun_out/r6e3; mkdir -p $O; export TMPDIR=/tmp PYTHONFAULTHANDLER=1
st() { echo "[r6e3] $(date +%T) $*"; }
for i in 1 2 3 4 5; do
  st run $i
  timeout -k 10 300 python -u bench/deploy_topology.py --kafka-replicated --kafka-controllers 3 --rate 1.2e6 \
    --seconds 60 --fmt json --log-dir $O/run$i --out $O/rf3_json_$i.json > $O/run$i.log 2>&1 \
    || { st "run $i failed"; tail -30 $O/run$i.log; exit 1; }
  python - $O/rf3_json_$i.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
cpu = {k: v for k, v in d["cpu_s_by_service"].items() if k.startswith("kafka")}
print("value", d["value"], "min", d["min_sample_tx_s"], "p2s", [(x["p50"], x["p99"]) for x in d["produce_to_scored_us"]],
      "checks", d["checks_passed"], "broker_cpu_s", cpu)
PY
done
st done
