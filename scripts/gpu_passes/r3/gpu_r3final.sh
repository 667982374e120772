#!/bin/bash
# Round-3 final regression of the exact committed tree: smoke, GPU suite, default benches.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3final
mkdir -p $O
step() { echo "[r3final] $(date +%T) $*"; }
step smoke
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
step pytest
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
step bench mlp
timeout -k 10 300 python bench.py --out $O/bench_mlp.json > $O/bench_mlp.log 2>&1 || { tail -30 $O/bench_mlp.log; exit 1; }
tail -1 $O/bench_mlp.log | cut -c1-400
step bench gbdt
timeout -k 10 300 python bench.py --model gbdt --out $O/bench_gbdt.json > $O/bench_gbdt.log 2>&1 || { tail -30 $O/bench_gbdt.log; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_gbdt.json')); print(d['value'], d['p50_latency_us'])"
step done
