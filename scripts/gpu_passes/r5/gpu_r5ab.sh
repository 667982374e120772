#!/usr/bin/env bash
# Round-5 pass AB (item 6): the 8-wave G20 build (two waves per SIMD) and the read-only build at the
# new grid range (216-240), against the default at 216.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 1
O=gpurun_out/r5ab; mkdir -p $O; export TMPDIR=/tmp
AB=ccfd_demo_summit_amd/_native/ab
st() { echo "[r5ab] $(date +%T) $*"; }
b() {   # b <name> <extra args> [env...]
  local n=$1 x=$2; shift 2
  st "$n"
  env "$@" timeout -k 10 240 python bench.py --model gbdt --steps 20 --warmup 5 $x > $O/$n.json 2> $O/$n.log \
    || { tail -30 $O/$n.log; exit 1; }
  python -c "import json; d=json.load(open('$O/$n.json')); p=d['precision_vs_fp32'] or {}; print('$n', d['value'], d['p50_latency_us'], d['p99_latency_us'], d['rows_scored'] == d['rows_expected'], d['wire_stale_rows'], p.get('route_flips_outside_1e-2_band'), p.get('max_abs_dp'))"
}
b default ""
b w8_g216 "--diagnostic --persist-grid 216" CCFD_LIB_PATH=$AB/w8.so
b w8_g240 "--diagnostic --persist-grid 240" CCFD_LIB_PATH=$AB/w8.so
b w8_g216_d5 "--diagnostic --persist-grid 216 --depth 5" CCFD_LIB_PATH=$AB/w8.so
b readonly_g216 "--diagnostic --persist-grid 216" CCFD_LIB_PATH=$AB/readonly.so
b default_d5 "--depth 5"
st done
