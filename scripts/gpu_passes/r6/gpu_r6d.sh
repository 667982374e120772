#!/usr/bin/env bash
# Round-6 pass D: the wave-specialised G20 loader kernel (CCFD_G32_LOADER=1, VGPR-staged rows,
# stop-aware waits) -- correctness, then config 4 loader vs default.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 1
O=gpurun_out/r6d; mkdir -p $O; export TMPDIR=/tmp PYTHONFAULTHANDLER=1
st() { echo "[r6d] $(date +%T) $*"; }
st pytest loader
CCFD_G32_LOADER=1 timeout -k 10 300 python -u -m pytest tests/test_gbdt_g20_gpu.py tests/test_handoff_lossless_gpu.py \
  -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_loader.log 2>&1 || { tail -40 $O/pytest_loader.log; exit 1; }
tail -1 $O/pytest_loader.log
for v in loader base loader256; do
  g=0
  case $v in base) e="CCFD_G32_LOADER=0";; loader) e="CCFD_G32_LOADER=1";; loader256) e="CCFD_G32_LOADER=1"; g=256;;
    loader128) e="CCFD_G32_LOADER=1"; g=128;; esac
  st bench $v
  env $e timeout -k 10 200 python -u bench.py --model gbdt --steps 20 --warmup 5 --diagnostic --watchdog-s 60 --persist-grid $g \
    > $O/bench_gbdt_$v.json 2> $O/bench_gbdt_$v.log || { st "bench $v failed"; tail -30 $O/bench_gbdt_$v.log; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['p50_latency_us'], d['p99_latency_us'], d['device_exec_us_mean'], d['precision_vs_fp32']['route_flips_outside_1e-2_band'], d['flagged_handed_off']==d['fraud_routed'])" $O/bench_gbdt_$v.json $v
done
st done
