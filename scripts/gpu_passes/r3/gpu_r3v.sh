#!/bin/bash
# Round-3 GPU pass V: compile-time A/B of the W64 fetch in the persistent claimed kernel --
# 16-byte lanes (default) vs 8-byte lanes + LDS hand-off (x2) vs 4-byte lanes + in-quad DPP
# transpose (q4); scripts/build_ab.py -> _native/ab/{x2,q4}.so; same box, alternating runs.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3v
mkdir -p $O
AB=$PWD/ccfd_demo_summit_amd/_native/ab
step() { echo "[r3v] $(date +%T) $*"; }
for v in x2 q4; do
  step pytest $v exactness
  CCFD_LIB_PATH=$AB/$v.so timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py tests/test_rules_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread -k "persistent" > $O/pytest_$v.log 2>&1 || { tail -40 $O/pytest_$v.log; exit 1; }
  tail -1 $O/pytest_$v.log
done
summ() { python3 -c "import json; d=json.load(open('$1')); r=d['per_rank'][0]; print('$1', '%.4g' % d['value'], 'p50', d['p50_latency_us'], 'p99', d.get('p99_latency_us'), 'h2d', r.get('h2d_zerocopy_GBps'), r.get('pci'), 'flips', d['precision_vs_fp32']['route_flips_outside_1e-2_band'])"; }
for i in 1 2 3; do
  step bench x4 $i
  timeout -k 10 300 python bench.py --min-timed-s 3 --out $O/x4_$i.json > $O/x4_$i.log 2>&1 || { tail -30 $O/x4_$i.log; exit 1; }
  summ $O/x4_$i.json
  for v in x2 q4; do
    step bench $v $i
    CCFD_LIB_PATH=$AB/$v.so timeout -k 10 300 python bench.py --min-timed-s 3 --out $O/${v}_$i.json > $O/${v}_$i.log 2>&1 || { tail -30 $O/${v}_$i.log; exit 1; }
    summ $O/${v}_$i.json
  done
done
step latency
for v in x4 x2 q4; do
  if [ $v = x4 ]; then unset CCFD_LIB_PATH; else export CCFD_LIB_PATH=$AB/$v.so; fi
  timeout -k 10 300 python bench/experiments/latency_breakdown.py --depths 1,8,12,16 --batches 3000 --out $O/lat_$v.jsonl > $O/lat_$v.log 2>&1 || { tail -20 $O/lat_$v.log; exit 1; }
done
unset CCFD_LIB_PATH
python3 - <<'PY'
import json
for v in ("x4", "x2", "q4"):
    for l in open(f"gpurun_out/r3v/lat_{v}.jsonl"):
        d = json.loads(l)
        print(v, "depth", d["depth"], "tx %.3g" % d["tx_s"], "p50", d["p50_total_us"], "dev", d["p50_dev_exec_us"])
PY
step done
