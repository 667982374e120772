#!/bin/bash
# Round-3 GPU pass P: regression of the whole tree after the round-3 kernel work -- smoke, the
# full GPU suite, the default bench, and a kernel-trace profile of the default bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3p
mkdir -p $O
step() { echo "[r3p] $(date +%T) $*"; }
step smoke
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
step pytest
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
step bench default
timeout -k 10 300 python bench.py --out $O/bench_default.json > $O/bench_default.log 2>&1 || { tail -30 $O/bench_default.log; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_default.json')); print(d['value'], d['p50_latency_us'], d['timed_region_s'])"
step rocprof kernel stats of the default bench
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 bench.py --out $O/bench_profiled.json > $O/prof.log 2>&1 || { tail -30 $O/prof.log; exit 1; }
find $O/prof -name "*kernel_stats.csv" | head -3
step done
