#!/bin/bash
# Round-3 GPU pass V: compile-time A/B of the W64 fetch (16-byte lanes vs 8-byte lanes + LDS
# hand-off, scripts/build_ab.py -> _native/ab/x2.so), same box, alternating runs.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3v
mkdir -p $O
X2=$PWD/ccfd_demo_summit_amd/_native/ab/x2.so
step() { echo "[r3v] $(date +%T) $*"; }
step pytest x2 exactness
CCFD_LIB_PATH=$X2 timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread -k "persistent" > $O/pytest_x2.log 2>&1 || { tail -40 $O/pytest_x2.log; exit 1; }
tail -1 $O/pytest_x2.log
summ() { python3 -c "import json; d=json.load(open('$1')); r=d['per_rank'][0]; print('$1', '%.4g' % d['value'], 'p50', d['p50_latency_us'], 'p99', d.get('p99_latency_us'), 'h2d', r.get('h2d_zerocopy_GBps'), r.get('pci'))"; }
for i in 1 2 3; do
  step bench x4 $i
  timeout -k 10 300 python bench.py --min-timed-s 3 --out $O/x4_$i.json > $O/x4_$i.log 2>&1 || { tail -30 $O/x4_$i.log; exit 1; }
  summ $O/x4_$i.json
  step bench x2 $i
  CCFD_LIB_PATH=$X2 timeout -k 10 300 python bench.py --min-timed-s 3 --out $O/x2_$i.json > $O/x2_$i.log 2>&1 || { tail -30 $O/x2_$i.log; exit 1; }
  summ $O/x2_$i.json
done
step latency
CCFD_LIB_PATH=$X2 timeout -k 10 300 python bench/experiments/latency_breakdown.py --depths 1,8,12,16 --batches 3000 --out $O/lat_x2.jsonl > $O/lat_x2.log 2>&1 || { tail -20 $O/lat_x2.log; exit 1; }
timeout -k 10 300 python bench/experiments/latency_breakdown.py --depths 1,8,12,16 --batches 3000 --out $O/lat_x4.jsonl > $O/lat_x4.log 2>&1 || { tail -20 $O/lat_x4.log; exit 1; }
python3 - <<'PY'
import json
for f in ("gpurun_out/r3v/lat_x2.jsonl", "gpurun_out/r3v/lat_x4.jsonl"):
    for l in open(f):
        d = json.loads(l)
        print(f[-10:-6], "depth", d["depth"], "tx %.3g" % d["tx_s"], "p50", d["p50_total_us"], "dev", d["p50_dev_exec_us"])
PY
step done
