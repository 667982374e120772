#!/bin/bash
# Round-3 GPU pass T: the final kernel tree (global-address-space hot loads / stores, dword
# G20 fetch): whole GPU suite, smoke, headline benches, kernel-trace profile.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${R3T_OUT:-r3t}
mkdir -p $O
step() { echo "[r3t] $(date +%T) $*"; }
step smoke
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
step pytest
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
summ() { python3 -c "import json; d=json.load(open('$1')); r=d['per_rank'][0]; print('$1', '%.4g' % d['value'], 'p50', d['p50_latency_us'], 'p99', d.get('p99_latency_us'), 'h2d', r.get('h2d_zerocopy_GBps'), r.get('pci'))"; }
for i in 1 2; do
  step bench mlp $i
  timeout -k 10 300 python bench.py --out $O/bench_mlp_$i.json > $O/bench_mlp_$i.log 2>&1 || { tail -30 $O/bench_mlp_$i.log; exit 1; }
  summ $O/bench_mlp_$i.json
done
step bench gbdt
timeout -k 10 300 python bench.py --model gbdt --out $O/bench_gbdt.json > $O/bench_gbdt.log 2>&1 || { tail -30 $O/bench_gbdt.log; exit 1; }
summ $O/bench_gbdt.json
step rocprof kernel stats
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 bench.py --out $O/bench_profiled.json > $O/prof.log 2>&1 || { tail -30 $O/prof.log; exit 1; }
summ $O/bench_profiled.json
step done
