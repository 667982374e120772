#!/usr/bin/env bash
# Round-6 pass E2: RF-3 JSON 1.2e6 tx/s produce -> scored tail, A/B of the follower fetcher
# (a task on the broker's event loop vs a thread per leader), of the controller (3-member
# quorum vs one process) and of the producers' request size (JSON messages per produce).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 1
O=gpurun_out/r6e2; mkdir -p $O; export TMPDIR=/tmp PYTHONFAULTHANDLER=1
st() { echo "[r6e2] $(date +%T) $*"; }
# cfg = <fetcher>-q<controllers>-b<producer batch: JSON messages per produce request>
for cfg in loop-q3-b1024 loop-q3-b4096 thread-q3-b1024 loop-q3-b2048 thread-q3-b4096; do
  mode=${cfg%%-*}; rest=${cfg#*-}; q=${rest%%-*}; q=${q#q}; b=${rest#*-b}; b=${b%x}
  st run $cfg
  CCFD_REPLICA_FETCH=$mode timeout -k 10 300 python -u bench/deploy_topology.py --kafka-replicated --kafka-controllers $q \
    --rate 1.2e6 --seconds 60 --fmt json --batch $b --log-dir $O/$cfg --out $O/rf3_json_$cfg.json > $O/$cfg.log 2>&1 \
    || { st "run $cfg failed"; tail -30 $O/$cfg.log; exit 1; }
  python - $O/rf3_json_$cfg.json $cfg <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
cpu = {k: v for k, v in d["cpu_s_by_service"].items() if k.startswith("kafka")}
print(sys.argv[2], "value", d["value"], "min", d["min_sample_tx_s"], "p2s", [(x["p50"], x["p99"]) for x in d["produce_to_scored_us"]],
      "checks", d["checks_passed"], "cpu", cpu)
PY
done
rm -rf $O/*/kafka-lite* 2>/dev/null
st done
