#!/usr/bin/env bash
# Round-5 pass I (VERDICT r4 items 4 + 6): the replicated kafka-lite after (a) replica fetches
# copying the log as appended and followers fetching again without waiting for their own write,
# (b) pipelined request handling per connection (responses in order), (c) service ports below
# the ephemeral range; RF 3 JSON with and without a broker SIGKILL, TXB1 with 8 producers at RF
# 3 and RF 1 and on the single-process broker.  Then the G20 item trace with the doorbell ring.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 1
O=gpurun_out/r5i; mkdir -p $O; export TMPDIR=/tmp PYTHONFAULTHANDLER=1
AB=ccfd_demo_summit_amd/_native/ab
st() { echo "[r5i] $(date +%T) $*"; }
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
        "arrival_to_scored_p99_us", "scrape_errors", "checks_passed")
print({k: d.get(k) for k in keys if k in d})
print("samples", [(s.get("tx_s"), s.get("under_replicated")) for s in d.get("samples", [])])
print("selectors", d.get("reference_dashboards", {}).get("matched"), "/", d.get("reference_dashboards", {}).get("selectors"))
PY
  return 0
}
R="python bench/deploy_topology.py --kafka-replicated --producer-acks -1 --producer-max-in-flight 5"
run repl_json_60s 300 $R --seconds 60 --producers 3 --rate 1.2e6 --fmt json --log-dir $O/rj --out $O/repl_json_60s.json
run repl_json_60s_kill 330 $R --seconds 60 --producers 3 --rate 1.2e6 --fmt json --kafka-kill-at 25 --kafka-down-s 5 \
    --kafka-kill-node 2 --log-dir $O/rjk --out $O/repl_json_60s_kill.json
run repl_txb1_p8_rf3 240 $R --seconds 30 --producers 8 --rate 0 --fmt txb1 --log-dir $O/rt3 --out $O/repl_txb1_p8_rf3.json
run repl_txb1_p8_rf1 240 $R --kafka-rf 1 --seconds 30 --producers 8 --rate 0 --fmt txb1 --log-dir $O/rt1 --out $O/repl_txb1_p8_rf1.json
run single_txb1_p8 240 python bench/deploy_topology.py --seconds 30 --producers 8 --rate 0 --fmt txb1 \
    --log-dir $O/st --out $O/single_txb1_p8.json
st itrace
timeout -k 10 240 env CCFD_LIB_PATH=$AB/itrace.so CCFD_ITEM_TRACE_OUT=$O/itrace python bench.py --model gbdt --steps 20 \
    --warmup 5 --diagnostic > $O/gbdt_itrace.json 2> $O/gbdt_itrace.log || { tail -20 $O/gbdt_itrace.log; exit 1; }
python bench/experiments/item_trace.py $O/itrace.0 --json $O/itrace_phases.json && rm -f $O/itrace.*
st dbw_itrace
timeout -k 10 240 env CCFD_LIB_PATH=$AB/dbw_itrace.so CCFD_ITEM_TRACE_OUT=$O/dbw_itrace python bench.py --model gbdt --steps 20 \
    --warmup 5 --diagnostic > $O/gbdt_dbw_itrace.json 2> $O/gbdt_dbw_itrace.log || { tail -20 $O/gbdt_dbw_itrace.log; exit 1; }
python bench/experiments/item_trace.py $O/dbw_itrace.0 --json $O/dbw_itrace_phases.json && rm -f $O/dbw_itrace.*
for v in default dbw default_again; do
  st gbdt_$v
  L=""; D=""; [ $v = dbw ] && { L="CCFD_LIB_PATH=$AB/dbw.so"; D=--diagnostic; }
  timeout -k 10 240 env $L python bench.py --model gbdt --steps 20 --warmup 5 $D > $O/gbdt_$v.json 2> $O/gbdt_$v.log \
    || { tail -20 $O/gbdt_$v.log; exit 1; }
  python -c "import json; d=json.load(open('$O/gbdt_$v.json')); print('$v', d['value'], d['p50_latency_us'], d['p99_latency_us'], d.get('precision_vs_fp32', {}).get('route_flips_outside_1e-2_band'), d.get('wire_stale_rows'))"
done
st done
