#!/usr/bin/env bash
# Round-5 pass K (rerun as K2: depth 16 and 32; follower fetches bounded to 8 MB): (item 4) the RF-3 broker SIGKILL run, 90 s, after the follower restart fix (a
# follower below its leader's log start restarts there); (item 6) the G20 item trace at depth 4
# and 8 with the per-batch straggler view (batch span, its last item).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 1
O=gpurun_out/${R5K_OUT:-r5k}; mkdir -p $O; export TMPDIR=/tmp PYTHONFAULTHANDLER=1
AB=ccfd_demo_summit_amd/_native/ab
st() { echo "[r5k] $(date +%T) $*"; }
for d in 16 32; do
  st itrace_d$d
  timeout -k 10 240 env CCFD_LIB_PATH=$AB/itrace.so CCFD_ITEM_TRACE_OUT=$O/itrace_d$d python bench.py --model gbdt --steps 20 \
      --warmup 5 --depth $d --diagnostic > $O/gbdt_itrace_d$d.json 2> $O/gbdt_itrace_d$d.log || { tail -20 $O/gbdt_itrace_d$d.log; exit 1; }
  python bench/experiments/item_trace.py $O/itrace_d$d.0 --json $O/itrace_d${d}_phases.json && rm -f $O/itrace_d$d.*
done
st repl_json_90s_kill
timeout -k 10 400 python bench/deploy_topology.py --kafka-replicated --producer-acks -1 --producer-max-in-flight 5 \
    --seconds 90 --producers 3 --rate 1.2e6 --fmt json --kafka-kill-at 25 --kafka-down-s 5 --kafka-kill-node 2 \
    --log-dir $O/rjk --out $O/repl_json_90s_kill.json > $O/repl_json_90s_kill.log 2>&1; rc=$?
st "repl rc=$rc"; [ $rc -ge 2 ] && { tail -30 $O/repl_json_90s_kill.log; exit $rc; }
python - $O/repl_json_90s_kill.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
keys = ("value", "min_sample_tx_s", "min_sample_ratio", "incoming_equals_produced", "kie_duplicates",
        "under_replicated_max", "under_replicated_final", "kafka_outage", "produce_to_scored_us", "scrape_errors",
        "cgroup_cpu", "checks_passed")
print({k: d.get(k) for k in keys if k in d})
print("samples", [(s.get("tx_s"), s.get("under_replicated")) for s in d.get("samples", [])])
PY
grep -h "replication:\|was below" $O/rjk/kafka-broker2-restarted.log | cut -c1-300 | head -12
st done
