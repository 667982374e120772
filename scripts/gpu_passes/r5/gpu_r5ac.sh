#!/usr/bin/env bash
# Round-5 pass AC (item 6): 1024-row G20 items (CCFD_PERSIST_ITEM_ROWS) at the larger grids.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 1
O=gpurun_out/r5ac; mkdir -p $O; export TMPDIR=/tmp
AB=ccfd_demo_summit_amd/_native/ab
st() { echo "[r5ac] $(date +%T) $*"; }
b() {   # b <name> <extra args> [env...]
  local n=$1 x=$2; shift 2
  st "$n"
  env "$@" timeout -k 10 240 python bench.py --model gbdt --steps 20 --warmup 5 $x > $O/$n.json 2> $O/$n.log \
    || { tail -30 $O/$n.log; exit 1; }
  python -c "import json; d=json.load(open('$O/$n.json')); p=d['precision_vs_fp32'] or {}; print('$n', d['value'], d['p50_latency_us'], d['p99_latency_us'], d['rows_scored'] == d['rows_expected'], d['wire_stale_rows'], p.get('route_flips_outside_1e-2_band'), p.get('max_abs_dp'))"
}
b default ""
b rows1024_g216 "--persist-grid 216" CCFD_PERSIST_ITEM_ROWS=1024
b rows1024_g256 "--persist-grid 256" CCFD_PERSIST_ITEM_ROWS=1024
b rows1024_g256_d5 "--persist-grid 256 --depth 5" CCFD_PERSIST_ITEM_ROWS=1024
b g224_d5 "--persist-grid 224 --depth 5"
st done
