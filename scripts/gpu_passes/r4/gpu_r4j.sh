#!/bin/bash
# Round 4 regression of the current tree: smoke, the whole GPU suite, config 2 / 4 benches,
# the dp2 rehearsal launch, and the deployed topology after the host-only codec library and
# the service warm-up (TXB1 open loop, JSON 1.2e6/s, process mode 2e5/s).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4j
mkdir -p $O
step() { echo "[r4j] $(date +%T) $*"; }
step smoke
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
step pytest gpu
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
step bench mlp
timeout -k 10 300 python bench.py --out $O/bench_mlp.json > $O/bench_mlp.log 2>&1 || { tail -30 $O/bench_mlp.log; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_mlp.json')); print(d['value'], d['p50_latency_us'], d['p99_latency_us'], d.get('precision_vs_fp32', {}).get('kernel'))"
step bench gbdt
timeout -k 10 300 python bench.py --model gbdt --out $O/bench_gbdt.json > $O/bench_gbdt.log 2>&1 || { tail -30 $O/bench_gbdt.log; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_gbdt.json')); print(d['value'], d['p50_latency_us'], d['p99_latency_us'])"
step bench dp2 rehearsal
timeout -k 10 400 python bench.py --gpus 2 --rehearsal --steps 10 --warmup 3 > $O/bench_dp2r.json 2> $O/bench_dp2r.log || { tail -30 $O/bench_dp2r.log; exit 1; }
cut -c1-300 $O/bench_dp2r.json
show() { python3 -c "
import json,sys; d=json.load(open(sys.argv[1]))
print(d['value'], d['min_sample_tx_s'], d['producers_tx_s'], 'arrival->scored', d['arrival_to_scored_p50_us'], d['arrival_to_scored_p99_us'], 'checks', d['checks_passed'], d.get('kie_standard_plus_fraud_equals_incoming'))
print('window', d.get('window_wall'), 'samples', [s['tx_s'] for s in d['samples']])
print('produce->scored', d['produce_to_scored_us'])
print('scored->started', d['scored_to_process_started_us'])
print('engine handoff', d.get('handoff_engine_us'))
print('kie', d.get('kie_handoff_attribution'))" "$1"; }
run() {
  local n=$1; shift
  step $n
  timeout -k 30 300 python bench/deploy_topology.py --seconds 30 "$@" --log-dir $O/$n --out $O/$n.json > $O/$n.log 2>&1 \
    || { tail -40 $O/$n.log; exit 1; }
  show $O/$n.json
}
run txb1 --producers 4 --rate 0 --fmt txb1
run json --producers 3 --rate 1200000 --fmt json
run json_process --producers 2 --rate 200000 --fmt json --standard-mode process
grep -h "native codecs loaded" $O/txb1/*.log | head -3
step done
