#!/bin/bash
# Round 4, the committed tree after the 3-way CRC-32C: smoke, the whole GPU suite, the default
# bench as the driver runs it, and the deployed topology (TXB1 with 4 and 8 producers, JSON).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4v
mkdir -p $O
step() { echo "[r4v] $(date +%T) $*"; }
step smoke
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
step pytest gpu
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
step bench default
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_default.json 2> $O/bench_default.log || { tail -30 $O/bench_default.log; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench_default.json').read().strip().splitlines()[-1]); print(d['value'], d['p50_latency_us'], d['p99_latency_us'])"
show() { python3 -c "
import json,sys; d=json.load(open(sys.argv[1]))
print(d['value'], d['min_sample_tx_s'], d['producers_tx_s'], 'checks', d['checks_passed'], 'a->s', d['arrival_to_scored_p50_us'], d['arrival_to_scored_p99_us'])
print('produce->scored', d['produce_to_scored_us']); print('scored->started', d['scored_to_process_started_us'])" "$1"; }
run() {
  local n=$1; shift
  step $n
  timeout -k 30 300 python bench/deploy_topology.py --seconds 30 "$@" --log-dir $O/$n --out $O/$n.json > $O/$n.log 2>&1 \
    || { tail -40 $O/$n.log; exit 1; }
  show $O/$n.json
}
run txb1_p4 --producers 4 --rate 0 --fmt txb1
run txb1_p8 --producers 8 --rate 0 --fmt txb1
run json --producers 3 --rate 1200000 --fmt json
step done
