#!/usr/bin/env bash
# Round-6 pass C: config-4 kernel variants -- the paired-chunk tree walk (CCFD_G32_PAIR) and the
# wave-specialised loader kernel (CCFD_G32_LOADER): correctness of the G20 / G32 persistent
# paths in each mode, then config 4 A/B/C twice each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 1
O=gpurun_out/r6c; mkdir -p $O; export TMPDIR=/tmp PYTHONFAULTHANDLER=1
st() { echo "[r6c] $(date +%T) $*"; }
for mode in "CCFD_G32_LOADER=1" "CCFD_G32_PAIR=1"; do
  st pytest $mode
  env $mode timeout -k 10 300 python -u -m pytest tests/test_gbdt_g20_gpu.py tests/test_gbdt_g32_gpu.py \
    tests/test_handoff_lossless_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_${mode%%=*}.log 2>&1 \
    || { tail -40 $O/pytest_${mode%%=*}.log; exit 1; }
  tail -1 $O/pytest_${mode%%=*}.log
done
for i in 1 2; do
  for v in base pair loader; do
    case $v in base) e="CCFD_G32_PAIR=0";; pair) e="CCFD_G32_PAIR=1";; loader) e="CCFD_G32_LOADER=1";; esac
    st bench $v run $i
    env $e timeout -k 10 300 python bench.py --model gbdt --steps 20 --warmup 5 --diagnostic \
      > $O/bench_gbdt_${v}_$i.json 2> $O/bench_gbdt_${v}_$i.log || { tail -30 $O/bench_gbdt_${v}_$i.log; exit 1; }
  done
done
python - $O <<'PY'
import json, sys, glob
for f in sorted(glob.glob(f"{sys.argv[1]}/bench_gbdt_*.json")):
    d = json.load(open(f))
    print(f.split("/")[-1], d["value"], d["p50_latency_us"], d["p99_latency_us"], "dev", d["device_exec_us_mean"],
          "flips", d["precision_vs_fp32"]["route_flips_outside_1e-2_band"], "handed", d["flagged_handed_off"] == d["fraud_routed"])
PY
st done
