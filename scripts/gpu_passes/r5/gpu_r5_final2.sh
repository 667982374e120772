#!/usr/bin/env bash
# Round-5 final pass 2: the committed tree after the G20 grid retune (216) and the kafka-lite
# callback responses / gathered sends -- GPU suite, smoke, config 2 / 4 as the driver runs them,
# and one deployed run per VERDICT r4 item: process mode on 4 KIE shards (1), the notification
# crash comparison (2), the 4-rank rehearsal with the trace, 2 HW queues per rank (3), and the
# replicated kafka-lite at RF 3: JSON 60 s, broker SIGKILL, TXB1 with 8 producers (4).  A deploy
# step whose checks fail (rc 1) does not stop the pass; a crash, abort or time limit does.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 1
O=gpurun_out/r5final2; mkdir -p $O; export TMPDIR=/tmp PYTHONFAULTHANDLER=1
st() { echo "[final2] $(date +%T) $*"; }
st pytest
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
st smoke
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
st bench
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_mlp.json 2> $O/bench_mlp.log || { tail -30 $O/bench_mlp.log; exit 1; }
timeout -k 10 300 python bench.py --model gbdt --steps 20 --warmup 5 > $O/bench_gbdt.json 2> $O/bench_gbdt.log || { tail -30 $O/bench_gbdt.log; exit 1; }
python - $O <<'PY'
import json, sys
for n in ("mlp", "gbdt"):
    d = json.load(open(f"{sys.argv[1]}/bench_{n}.json"))
    p = d["precision_vs_fp32"]
    print(n, d["value"], d["p50_latency_us"], d["p99_latency_us"], "flips", p["route_flips_outside_1e-2_band"],
          "ceiling", d["h2d_zerocopy_ceiling_tx_s_rank0"], d["config"]["parallelism"])
PY
run() {   # run <name> <seconds> <cmd...>
  local n=$1 t=$2; shift 2
  st "$n"
  timeout -k 10 "$t" "$@" > $O/$n.log 2>&1; local rc=$?
  st "$n rc=$rc"
  if [ $rc -ne 0 ]; then grep "\[deploy\]" $O/$n.log | tail -5; tail -15 $O/$n.log; fi
  if [ $rc -ge 2 ]; then exit $rc; fi
  [ -f $O/$n.json ] && python - $O/$n.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
keys = ("value", "min_sample_tx_s", "min_sample_ratio", "incoming_equals_produced", "kie_standard_plus_fraud_equals_incoming",
        "kie_duplicates", "under_replicated_max", "under_replicated_final", "scored_to_process_started_us",
        "produce_to_scored_us", "arrival_to_scored_p99_us", "same_outcomes_as", "checks_passed")
print({k: d.get(k) for k in keys if k in d})
print("selectors", d.get("reference_dashboards", {}).get("matched"), "/", d.get("reference_dashboards", {}).get("selectors"))
PY
  return 0
}
D="python bench/deploy_topology.py"
run process_k4_60s 330 $D --standard-mode process --kie-shards 4 --rate 1.2e6 --producers 3 --fmt json --seconds 60 \
    --log-dir $O/p60 --out $O/process_k4_60s.json
N="$D --kie-shards 2 --rate 1.0e6 --producers 2 --fmt json --count 10000000 --seconds 30 --settle --notification-timeout-s 20 --notifier-seed 7"
run notif_ref 300 $N --log-dir $O/nref --out $O/notif_ref.json
run notif_crash 330 $N --kie-outage-at 8 --kie-kill-shard 0 --kie-outage-s 3 --notifier-kill-at 11 --notifier-down-s 3 \
    --compare-to $O/notif_ref.json --log-dir $O/ncrash --out $O/notif_crash.json
R="$D --kafka-replicated --producer-acks -1 --producer-max-in-flight 5"
run repl_json_90s_kill 400 $R --seconds 90 --producers 3 --rate 1.2e6 --fmt json --kafka-kill-at 25 --kafka-down-s 5 \
    --kafka-kill-node 2 --log-dir $O/rjk --out $O/repl_json_90s_kill.json
run repl_json_60s 300 $R --seconds 60 --producers 3 --rate 1.2e6 --fmt json --log-dir $O/rj --out $O/repl_json_60s.json
run repl_txb1_p8_rf3 240 $R --seconds 30 --producers 8 --rate 0 --fmt txb1 --log-dir $O/rt3 --out $O/repl_txb1_p8_rf3.json
run topo4_count 300 $D --ranks 4 --rehearsal --seconds 20 --producers 3 --rate 600000 --fmt json --trace \
    --log-dir $O/t4c --out $O/topo4_count.json
run topo4_process 300 $D --ranks 4 --rehearsal --seconds 20 --producers 3 --rate 600000 --fmt json --trace \
    --standard-mode process --kie-shards 4 --log-dir $O/t4p --out $O/topo4_process.json
for t in t4c t4p; do
  [ -d $O/$t/service_trace ] && python bench/tail_attribution.py $O/$t/service_trace/rank*.npz --out $O/${t}_tail.json > /dev/null \
    && python -c "import json; [print('$t', r['trace'][-9:], r['arrival_to_landed_us']['p99'], r['device_start_wait_us'], r['device_stall_windows']) for r in json.load(open('$O/${t}_tail.json'))]"
done
rm -rf $O/p60 $O/nref $O/ncrash $O/rjk $O/rj $O/rt3
find $O/t4c $O/t4p -name "*.npz" -delete 2>/dev/null
st done
