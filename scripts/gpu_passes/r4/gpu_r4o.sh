#!/bin/bash
# Round 4 final regression of the committed tree: smoke, the whole GPU suite, config 2 / 4
# benches; then the deployed topology (durable write-behind broker with the short GIL switch
# interval) against the in-memory broker on the same box, JSON parse threads 1 vs 4, and the
# process mode.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4o
mkdir -p $O
step() { echo "[r4o] $(date +%T) $*"; }
step smoke
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
step pytest gpu
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
step bench mlp
timeout -k 10 300 python bench.py --out $O/bench_mlp.json > $O/bench_mlp.log 2>&1 || { tail -30 $O/bench_mlp.log; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_mlp.json')); print(d['value'], d['p50_latency_us'], d['p99_latency_us'])"
step bench gbdt
timeout -k 10 300 python bench.py --model gbdt --out $O/bench_gbdt.json > $O/bench_gbdt.log 2>&1 || { tail -30 $O/bench_gbdt.log; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_gbdt.json')); print(d['value'], d['p50_latency_us'], d['p99_latency_us'])"
show() { python3 -c "
import json,sys; d=json.load(open(sys.argv[1]))
print(d['value'], d['min_sample_tx_s'], d['producers_tx_s'], 'a->s', d['arrival_to_scored_p50_us'], d['arrival_to_scored_p99_us'], 'checks', d['checks_passed'], d.get('kie_standard_plus_fraud_equals_incoming'), 'durable', d.get('kafka_durable'))
print('produce->scored', d['produce_to_scored_us'])
print('scored->started', d['scored_to_process_started_us'])" "$1"; }
run() {
  local n=$1; shift
  step $n
  timeout -k 30 300 python bench/deploy_topology.py --seconds 30 "$@" --log-dir $O/$n --out $O/$n.json > $O/$n.log 2>&1 \
    || { tail -40 $O/$n.log; exit 1; }
  show $O/$n.json
}
run txb1_durable --producers 4 --rate 0 --fmt txb1
run txb1_memory --producers 4 --rate 0 --fmt txb1 --kafka-memory
run json_durable --producers 3 --rate 1200000 --fmt json
run json_memory --producers 3 --rate 1200000 --fmt json --kafka-memory
CCFD_KC_PARSE_THREADS=4 run json_durable_p4 --producers 3 --rate 1200000 --fmt json
run json_process --producers 2 --rate 200000 --fmt json --standard-mode process
step done
