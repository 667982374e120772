#!/bin/bash
# Round 4: the G20 two-item pipeline (CCFD_G32_ITEM_PREFETCH) -- exactness, then config-4
# A/B against the default; config 5 TXB1 open loop (4 producers, native serving) and the
# process-mode run again after the GC policy / binary standard hand-off.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4f
mkdir -p $O
step() { echo "[r4f] $(date +%T) $*"; }
step pytest item prefetch
timeout -k 10 300 python -u -m pytest tests/test_gbdt_g20_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread \
  -k "item_prefetch or persistent_partial" > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
summ() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], '%.4g tx/s' % d['value'], 'p50', d['p50_latency_us'], 'p99', d['p99_latency_us'])" "$1" "$2"; }
for rep in 1 2; do
  step gbdt default rep $rep
  timeout -k 10 300 python bench.py --model gbdt --out $O/gbdt_default_$rep.json > $O/gbdt_default_$rep.log 2>&1 || { tail -30 $O/gbdt_default_$rep.log; exit 1; }
  summ $O/gbdt_default_$rep.json default
  step gbdt item prefetch rep $rep
  CCFD_G32_ITEM_PREFETCH=1 timeout -k 10 300 python bench.py --model gbdt --out $O/gbdt_prefetch_$rep.json > $O/gbdt_prefetch_$rep.log 2>&1 || { tail -30 $O/gbdt_prefetch_$rep.log; exit 1; }
  summ $O/gbdt_prefetch_$rep.json prefetch
done
for g in 128 256; do
  step gbdt item prefetch grid $g
  CCFD_G32_ITEM_PREFETCH=1 timeout -k 10 300 python bench.py --model gbdt --persist-grid $g --out $O/gbdt_prefetch_grid$g.json > $O/gbdt_prefetch_grid$g.log 2>&1 || { tail -30 $O/gbdt_prefetch_grid$g.log; exit 1; }
  summ $O/gbdt_prefetch_grid$g.json prefetch_grid$g
done
step gbdt item prefetch 256-row items
CCFD_G32_ITEM_PREFETCH=1 CCFD_PERSIST_ITEM_ROWS=256 timeout -k 10 300 python bench.py --model gbdt --out $O/gbdt_prefetch_item256.json > $O/gbdt_prefetch_item256.log 2>&1 || { tail -30 $O/gbdt_prefetch_item256.log; exit 1; }
summ $O/gbdt_prefetch_item256.json prefetch_item256
step txb1 open loop, 4 producers, native serving
timeout -k 30 300 python bench/deploy_topology.py --seconds 30 --producers 4 --rate 0 --fmt txb1 \
  --log-dir $O/txb1 --out $O/topo_txb1_4p.json > $O/topo_txb1_4p.log 2>&1 || { tail -40 $O/topo_txb1_4p.log; exit 1; }
python3 -c "import json; d=json.load(open('$O/topo_txb1_4p.json')); print(d['value'], d['min_sample_tx_s'], d['producers_tx_s'], d['arrival_to_scored_p50_us'], d['arrival_to_scored_p99_us'], d['produce_to_scored_us'], d['scored_to_process_started_us'], d['checks_passed']); print(d.get('handoff_engine_us'), d.get('kie_handoff_attribution'))"
step json process mode 2e5
timeout -k 30 300 python bench/deploy_topology.py --seconds 30 --producers 2 --rate 200000 --fmt json \
  --standard-mode process --log-dir $O/json_proc --out $O/topo_json_process.json > $O/topo_json_process.log 2>&1 || { tail -40 $O/topo_json_process.log; exit 1; }
python3 -c "import json; d=json.load(open('$O/topo_json_process.json')); print(d['value'], d['checks_passed'], d.get('kie_standard_plus_fraud_equals_incoming'), d['scored_to_process_started_us'], d['produce_to_scored_us'], d['arrival_to_scored_p99_us']); print(d.get('handoff_engine_us'), d.get('kie_handoff_attribution'))"
step done
