#!/usr/bin/env bash
# Round-5 pass U (item 6): claim-ahead G20 items (CCFD_EXP_CLAIM_AHEAD) -- before an item's last
# chunk is scored, claim the next item and put its first chunk's zero-copy load in flight --
# against the default claimed kernel, at ring depth 4 / 6 / 8.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 1
O=gpurun_out/r5u; mkdir -p $O; export TMPDIR=/tmp
AB=ccfd_demo_summit_amd/_native/ab
st() { echo "[r5u] $(date +%T) $*"; }
b() {   # b <name> <extra args> [env...]
  local n=$1 x=$2; shift 2
  st "$n"
  env "$@" timeout -k 10 240 python bench.py --model gbdt --steps 20 --warmup 5 $x > $O/$n.json 2> $O/$n.log \
    || { tail -30 $O/$n.log; exit 1; }
  python -c "import json; d=json.load(open('$O/$n.json')); p=d['precision_vs_fp32'] or {}; print('$n', d['value'], d['p50_latency_us'], d['p99_latency_us'], d['rows_scored'] == d['rows_expected'], d['wire_stale_rows'], p.get('route_flips_outside_1e-2_band'), p.get('max_abs_dp'))"
}
b default ""
b ahead "--diagnostic" CCFD_LIB_PATH=$AB/ahead.so
b ahead_d6 "--diagnostic --depth 6" CCFD_LIB_PATH=$AB/ahead.so
b ahead_d8 "--diagnostic --depth 8" CCFD_LIB_PATH=$AB/ahead.so
b default2 ""
b ahead2 "--diagnostic" CCFD_LIB_PATH=$AB/ahead.so
st done
