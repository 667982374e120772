#!/bin/bash
# Round-3 GPU pass Z: compile-time A/B of the G20 fetch (dword lanes, default, vs 16-byte
# lanes, _native/ab/g20x4.so), plus the default tree's smoke and GPU suite.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3z
mkdir -p $O
V=$PWD/ccfd_demo_summit_amd/_native/ab/g20x4.so
step() { echo "[r3z] $(date +%T) $*"; }
step smoke
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
step pytest default
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
step pytest g20x4 exactness
CCFD_LIB_PATH=$V timeout -k 10 300 python -u -m pytest tests/test_gbdt_g20_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_g20x4.log 2>&1 || { tail -40 $O/pytest_g20x4.log; exit 1; }
tail -1 $O/pytest_g20x4.log
summ() { python3 -c "import json; d=json.load(open('$1')); r=d['per_rank'][0]; print('$1', '%.4g' % d['value'], 'p50', d['p50_latency_us'], 'p99', d.get('p99_latency_us'), 'h2d', r.get('h2d_zerocopy_GBps'), 'flips', d['precision_vs_fp32']['route_flips'])"; }
for i in 1 2 3; do
  step gbdt dword $i
  timeout -k 10 200 python bench.py --model gbdt --min-timed-s 3 --out $O/dw_$i.json > $O/dw_$i.log 2>&1 || { tail -30 $O/dw_$i.log; exit 1; }
  summ $O/dw_$i.json
  step gbdt x4 $i
  CCFD_LIB_PATH=$V timeout -k 10 200 python bench.py --model gbdt --min-timed-s 3 --out $O/x4_$i.json > $O/x4_$i.log 2>&1 || { tail -30 $O/x4_$i.log; exit 1; }
  summ $O/x4_$i.json
done
step done
