#!/usr/bin/env bash
# Round-5 pass L (item 6): the item trace with the claim stamped when the atomic's value is back
# (the earlier traces stamped its issue), and per-XCD claim counters (CCFD_EXP_XCD_QUEUES).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 1
O=gpurun_out/r5l; mkdir -p $O; export TMPDIR=/tmp
AB=ccfd_demo_summit_amd/_native/ab
st() { echo "[r5l] $(date +%T) $*"; }
b() {   # b <name> <extra args> [env...]
  local n=$1 x=$2; shift 2
  st "$n"
  env "$@" timeout -k 10 240 python bench.py --model gbdt --steps 20 --warmup 5 $x > $O/$n.json 2> $O/$n.log \
    || { tail -30 $O/$n.log; exit 1; }
  python -c "import json; d=json.load(open('$O/$n.json')); print('$n', d['value'], d['p50_latency_us'], d['p99_latency_us'], d.get('precision_vs_fp32', {}).get('route_flips_outside_1e-2_band'), d.get('wire_stale_rows'), d['rows_scored'] == d['rows_expected'])"
}
b default ""
b itrace --diagnostic CCFD_LIB_PATH=$AB/itrace.so CCFD_ITEM_TRACE_OUT=$O/itrace
python bench/experiments/item_trace.py $O/itrace.0 --json $O/itrace_phases.json && rm -f $O/itrace.*
b xcdq_g193 "--diagnostic --persist-grid 193" CCFD_LIB_PATH=$AB/xcdq.so
b xcdq_g192 "--diagnostic --persist-grid 192" CCFD_LIB_PATH=$AB/xcdq.so
b xcdq_g257 "--diagnostic --persist-grid 257" CCFD_LIB_PATH=$AB/xcdq.so
b default_again ""
st done
