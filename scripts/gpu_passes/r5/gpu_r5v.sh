#!/usr/bin/env bash
# Round-5 pass V (item 6): run-time operating points of the default G20 kernel -- the whole
# item in flight (CCFD_G32_INFLIGHT=1), 256-row items, depth 5, grids 161 / 224.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 1
O=gpurun_out/r5v; mkdir -p $O; export TMPDIR=/tmp
AB=ccfd_demo_summit_amd/_native/ab
st() { echo "[r5v] $(date +%T) $*"; }
b() {   # b <name> <extra args> [env...]
  local n=$1 x=$2; shift 2
  st "$n"
  env "$@" timeout -k 10 240 python bench.py --model gbdt --steps 20 --warmup 5 $x > $O/$n.json 2> $O/$n.log \
    || { tail -30 $O/$n.log; exit 1; }
  python -c "import json; d=json.load(open('$O/$n.json')); p=d['precision_vs_fp32'] or {}; print('$n', d['value'], d['p50_latency_us'], d['p99_latency_us'], d['rows_scored'] == d['rows_expected'], d['wire_stale_rows'], p.get('route_flips_outside_1e-2_band'), p.get('max_abs_dp'))"
}
b default ""
b inflight "" CCFD_G32_INFLIGHT=1
b inflight_d5 "--depth 5" CCFD_G32_INFLIGHT=1
b d5 "--depth 5"
b rows256 "" CCFD_PERSIST_ITEM_ROWS=256
b rows256_d5 "--depth 5" CCFD_PERSIST_ITEM_ROWS=256
b grid224 "--persist-grid 224"
b grid161 "--persist-grid 161"
st done
