#!/usr/bin/env bash
# Round-5 pass AA (item 4): the native consumer parsing JSON produce requests 1024 records at a
# time -- RF-3 JSON 60 s (fetched -> scored gap) and the single durable broker JSON 60 s.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 1
O=gpurun_out/r5aa; mkdir -p $O; export TMPDIR=/tmp PYTHONFAULTHANDLER=1
st() { echo "[r5aa] $(date +%T) $*"; }
run() {   # run <name> <seconds> <cmd...>
  local n=$1 t=$2; shift 2
  st "$n"
  timeout -k 10 "$t" "$@" > $O/$n.log 2>&1; local rc=$?
  st "$n rc=$rc"
  if [ $rc -ne 0 ]; then grep "\[deploy\]" $O/$n.log | tail -8; tail -25 $O/$n.log; fi
  if [ $rc -ge 2 ]; then exit $rc; fi
  [ -f $O/$n.json ] && python - $O/$n.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
keys = ("value", "min_sample_tx_s", "min_sample_ratio", "incoming_equals_produced", "kie_duplicates",
        "under_replicated_max", "under_replicated_final", "kafka_outage", "produce_to_scored_us",
        "arrival_to_scored_p99_us", "scrape_errors", "cgroup_cpu", "checks_passed")
print({k: d.get(k) for k in keys if k in d})
print("samples", [(s.get("tx_s"), s.get("under_replicated")) for s in d.get("samples", [])])
PY
  return 0
}
R="python bench/deploy_topology.py --kafka-replicated --producer-acks -1 --producer-max-in-flight 5"
run repl_json_60s 300 $R --seconds 60 --producers 3 --rate 1.2e6 --fmt json --log-dir $O/rj --out $O/repl_json_60s.json
run json_60s 300 python bench/deploy_topology.py --seconds 60 --producers 3 --rate 1.2e6 --fmt json --log-dir $O/sj \
    --out $O/json_60s.json
rm -rf $O/rj $O/sj
st done
