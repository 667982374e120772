#!/usr/bin/env bash
# Round-5 pass Q (item 6): bigger G20 items -- 1024 rows (40 KB of input: the W64 MLP's items
# are 32 KB) -- with 8 waves (two chunks each) and with the default 4 (four chunks each).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 1
O=gpurun_out/r5q; mkdir -p $O; export TMPDIR=/tmp
AB=ccfd_demo_summit_amd/_native/ab
st() { echo "[r5q] $(date +%T) $*"; }
b() {   # b <name> <extra args> [env...]
  local n=$1 x=$2; shift 2
  st "$n"
  env "$@" timeout -k 10 240 python bench.py --model gbdt --steps 20 --warmup 5 $x > $O/$n.json 2> $O/$n.log \
    || { tail -30 $O/$n.log; exit 1; }
  python -c "import json; d=json.load(open('$O/$n.json')); print('$n', d['value'], d['p50_latency_us'], d['p99_latency_us'], d.get('precision_vs_fp32', {}).get('route_flips_outside_1e-2_band'), d.get('wire_stale_rows'), d['rows_scored'] == d['rows_expected'])"
}
b default ""
b w8_i1024 "--diagnostic" CCFD_LIB_PATH=$AB/w8.so CCFD_PERSIST_ITEM_ROWS=1024
b w8_i1024_g129 "--diagnostic --persist-grid 129" CCFD_LIB_PATH=$AB/w8.so CCFD_PERSIST_ITEM_ROWS=1024
b i1024 "" CCFD_PERSIST_ITEM_ROWS=1024
b w8_i1024_d6 "--diagnostic --depth 6" CCFD_LIB_PATH=$AB/w8.so CCFD_PERSIST_ITEM_ROWS=1024
st done
