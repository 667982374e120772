#!/bin/bash
# Round-3 GPU pass S: 8-byte-lane W64 fetch (CCFD_W64_FETCH_X2) exactness + same-box A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3s
mkdir -p $O
step() { echo "[r3s] $(date +%T) $*"; }
step pytest
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py tests/test_gbdt_g20_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
summ() { python3 -c "import json; d=json.load(open('$1')); print('$1', '%.4g' % d['value'], 'p50', d['p50_latency_us'], 'p99', d.get('p99_latency_us'), 'dev', d['device_exec_us_p50'], 't', d['timed_region_s'])"; }
for i in 1 2; do
  step bench default $i
  timeout -k 10 300 python bench.py --out $O/bench_x4_$i.json > $O/bench_x4_$i.log 2>&1 || { tail -30 $O/bench_x4_$i.log; exit 1; }
  summ $O/bench_x4_$i.json
  step bench x2 $i
  CCFD_W64_FETCH_X2=1 timeout -k 10 300 python bench.py --out $O/bench_x2_$i.json > $O/bench_x2_$i.log 2>&1 || { tail -30 $O/bench_x2_$i.log; exit 1; }
  summ $O/bench_x2_$i.json
done
step bench gbdt dword default
timeout -k 10 300 python bench.py --model gbdt --out $O/bench_gbdt.json > $O/bench_gbdt.log 2>&1 || { tail -30 $O/bench_gbdt.log; exit 1; }
summ $O/bench_gbdt.json
step latency x2
CCFD_W64_FETCH_X2=1 timeout -k 10 300 python bench/experiments/latency_breakdown.py --depths 1,4,8,12 --batches 3000 --out $O/lat_x2.jsonl > $O/lat_x2.log 2>&1 || { tail -20 $O/lat_x2.log; exit 1; }
timeout -k 10 300 python bench/experiments/latency_breakdown.py --depths 1,4,8,12 --batches 3000 --out $O/lat_x4.jsonl > $O/lat_x4.log 2>&1 || { tail -20 $O/lat_x4.log; exit 1; }
python3 - <<'PY'
import json
for f in ("gpurun_out/r3s/lat_x2.jsonl", "gpurun_out/r3s/lat_x4.jsonl"):
    for l in open(f):
        d = json.loads(l)
        print(f[-10:-6], "depth", d["depth"], "tx %.3g" % d["tx_s"], "p50", d["p50_total_us"], "dev", d["p50_dev_exec_us"])
PY
step done
