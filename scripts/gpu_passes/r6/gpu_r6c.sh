#!/usr/bin/env bash
# Round-6 pass C: paired-chunk tree walk (CCFD_G32_PAIR) -- correctness of the G20/G32
# persistent kernels in that mode, then config 4 A/B (default vs pair) twice each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 1
O=gpurun_out/r6c; mkdir -p $O; export TMPDIR=/tmp PYTHONFAULTHANDLER=1
st() { echo "[r6c] $(date +%T) $*"; }
st pytest pair
CCFD_G32_PAIR=1 timeout -k 10 600 python -u -m pytest tests/test_gbdt_g20_gpu.py tests/test_gbdt_g32_gpu.py \
  tests/test_handoff_lossless_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_pair.log 2>&1 \
  || { tail -40 $O/pytest_pair.log; exit 1; }
tail -1 $O/pytest_pair.log
for i in 1 2; do
  for v in 0 1; do
    st bench pair=$v run $i
    CCFD_G32_PAIR=$v timeout -k 10 300 python bench.py --model gbdt --steps 20 --warmup 5 --diagnostic \
      > $O/bench_gbdt_pair${v}_$i.json 2> $O/bench_gbdt_pair${v}_$i.log || { tail -30 $O/bench_gbdt_pair${v}_$i.log; exit 1; }
  done
done
python - $O <<'PY'
import json, sys, glob
for f in sorted(glob.glob(f"{sys.argv[1]}/bench_gbdt_pair*.json")):
    d = json.load(open(f))
    print(f.split("/")[-1], d["value"], d["p50_latency_us"], d["p99_latency_us"], "dev", d["device_exec_us_mean"],
          "flips", d["precision_vs_fp32"]["route_flips_outside_1e-2_band"], "handed", d["flagged_handed_off"] == d["fraud_routed"])
PY
st done
