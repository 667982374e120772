#!/bin/bash
# Round 4: last regression of the committed tree -- smoke, the whole GPU suite, config 2 / 4
# benches exactly as the driver runs them, and one deployed JSON run.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4r
mkdir -p $O
step() { echo "[r4r] $(date +%T) $*"; }
step smoke
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
step pytest gpu
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
step bench default
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_default.json 2> $O/bench_default.log || { tail -30 $O/bench_default.log; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench_default.json').read().strip().splitlines()[-1]); print(d['value'], d['p50_latency_us'], d['p99_latency_us'], d['ms_per_step'])"
step bench gbdt
timeout -k 10 300 python bench.py --model gbdt --out $O/bench_gbdt.json > $O/bench_gbdt.log 2>&1 || { tail -30 $O/bench_gbdt.log; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_gbdt.json')); print(d['value'], d['p50_latency_us'], d['p99_latency_us'])"
step json topology
timeout -k 30 300 python bench/deploy_topology.py --seconds 30 --producers 3 --rate 1200000 --fmt json \
  --log-dir $O/json --out $O/json.json > $O/json.log 2>&1 || { tail -40 $O/json.log; exit 1; }
python3 -c "
import json; d=json.load(open('$O/json.json'))
print(d['value'], d['min_sample_tx_s'], d['checks_passed'], d['arrival_to_scored_p50_us'], d['arrival_to_scored_p99_us'])
print(d['produce_to_scored_us']); print(d['scored_to_process_started_us'])"
step done
