#!/bin/bash
# Round 4: the G20 kernel after removing the prefetch variant (tests + config 4), then the
# deployed topology with the scored -> started attribution (engine hand-off + KIE) and the
# produce -> scored split (send -> fetched at the consumer): TXB1 open loop, JSON at 1.2e6/s,
# process mode at 2e5/s.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4g
mkdir -p $O
step() { echo "[r4g] $(date +%T) $*"; }
step pytest g20
timeout -k 10 300 python -u -m pytest tests/test_gbdt_g20_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread \
  > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
step gbdt default
timeout -k 10 300 python bench.py --model gbdt --out $O/gbdt_default.json > $O/gbdt_default.log 2>&1 || { tail -30 $O/gbdt_default.log; exit 1; }
python3 -c "import json; d=json.load(open('$O/gbdt_default.json')); print(d['value'], d['p50_latency_us'], d['p99_latency_us'])"
show() { python3 -c "
import json,sys; d=json.load(open(sys.argv[1]))
print(d['value'], d['min_sample_tx_s'], d['producers_tx_s'], 'arrival->scored', d['arrival_to_scored_p50_us'], d['arrival_to_scored_p99_us'], 'checks', d['checks_passed'], d.get('kie_standard_plus_fraud_equals_incoming'))
print('produce->scored', d['produce_to_scored_us'])
print('scored->started', d['scored_to_process_started_us'])
print('engine handoff', d.get('handoff_engine_us'))
print('kie', d.get('kie_handoff_attribution'))" "$1"; }
step txb1 open loop, 4 producers
timeout -k 30 300 python bench/deploy_topology.py --seconds 30 --producers 4 --rate 0 --fmt txb1 \
  --log-dir $O/txb1 --out $O/topo_txb1_4p.json > $O/topo_txb1_4p.log 2>&1 || { tail -40 $O/topo_txb1_4p.log; exit 1; }
show $O/topo_txb1_4p.json
step json 1.2e6
timeout -k 30 300 python bench/deploy_topology.py --seconds 30 --producers 3 --rate 1200000 --fmt json \
  --log-dir $O/json --out $O/topo_json.json > $O/topo_json.log 2>&1 || { tail -40 $O/topo_json.log; exit 1; }
show $O/topo_json.json
step json process mode 2e5
timeout -k 30 300 python bench/deploy_topology.py --seconds 30 --producers 2 --rate 200000 --fmt json \
  --standard-mode process --log-dir $O/json_proc --out $O/topo_json_process.json > $O/topo_json_process.log 2>&1 || { tail -40 $O/topo_json_process.log; exit 1; }
show $O/topo_json_process.json
step done
