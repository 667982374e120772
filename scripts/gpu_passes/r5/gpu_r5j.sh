#!/usr/bin/env bash
# Round-5 pass J: (item 4) the RF-3 broker SIGKILL run again, 90 s so the restarted broker has
# time to catch up, with the brokers' replication status lines (fetch rate, how far behind, ISR,
# fetch errors) and the HW checkpoint off the event loop; the RF-3 JSON run without a kill; the
# cgroup CPU-throttling counters and per-service CPU of each run.  (Item 6) the G20 item +
# doorbell trace at depth 8.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 1
O=gpurun_out/r5j; mkdir -p $O; export TMPDIR=/tmp PYTHONFAULTHANDLER=1
AB=ccfd_demo_summit_amd/_native/ab
st() { echo "[r5j] $(date +%T) $*"; }
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
        "arrival_to_scored_p99_us", "scrape_errors", "cgroup_cpu", "cpu_s_by_service", "checks_passed")
print({k: d.get(k) for k in keys if k in d})
print("samples", [(s.get("tx_s"), s.get("under_replicated")) for s in d.get("samples", [])])
PY
  return 0
}
R="python bench/deploy_topology.py --kafka-replicated --producer-acks -1 --producer-max-in-flight 5"
run repl_json_90s_kill 400 $R --seconds 90 --producers 3 --rate 1.2e6 --fmt json --kafka-kill-at 25 --kafka-down-s 5 \
    --kafka-kill-node 2 --log-dir $O/rjk --out $O/repl_json_90s_kill.json
grep -h "replication:" $O/rjk/kafka-broker2-restarted.log | cut -c1-400 | tail -12
run repl_json_60s 300 $R --seconds 60 --producers 3 --rate 1.2e6 --fmt json --log-dir $O/rj --out $O/repl_json_60s.json
st itrace_d8
timeout -k 10 240 env CCFD_LIB_PATH=$AB/itrace.so CCFD_ITEM_TRACE_OUT=$O/itrace_d8 python bench.py --model gbdt --steps 20 \
    --warmup 5 --depth 8 --diagnostic > $O/gbdt_itrace_d8.json 2> $O/gbdt_itrace_d8.log || { tail -20 $O/gbdt_itrace_d8.log; exit 1; }
python bench/experiments/item_trace.py $O/itrace_d8.0 --json $O/itrace_d8_phases.json && rm -f $O/itrace_d8.*
st done
