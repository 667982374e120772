#!/usr/bin/env bash
# Round-5 pass W (item 6): the default G20 kernel across persistent grids 193..249 at depth 4
# (pass V: grid 224 measured 2.55e9 against 2.53e9 at the default 192).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 1
O=gpurun_out/r5w; mkdir -p $O; export TMPDIR=/tmp
AB=ccfd_demo_summit_amd/_native/ab
st() { echo "[r5w] $(date +%T) $*"; }
b() {   # b <name> <extra args> [env...]
  local n=$1 x=$2; shift 2
  st "$n"
  env "$@" timeout -k 10 240 python bench.py --model gbdt --steps 20 --warmup 5 $x > $O/$n.json 2> $O/$n.log \
    || { tail -30 $O/$n.log; exit 1; }
  python -c "import json; d=json.load(open('$O/$n.json')); p=d['precision_vs_fp32'] or {}; print('$n', d['value'], d['p50_latency_us'], d['p99_latency_us'], d['rows_scored'] == d['rows_expected'], d['wire_stale_rows'], p.get('route_flips_outside_1e-2_band'), p.get('max_abs_dp'))"
}
for g in 192 200 208 216 224 232 240 249 224 216; do b g$g "--persist-grid $g"; done
st done
