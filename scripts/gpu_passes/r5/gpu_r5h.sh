#!/usr/bin/env bash
# Round-5 pass H (second step): the item trace with the posting wait split
# from the descriptor read, the cost of the per-item agent-scope acquire (CCFD_EXP_NO_ACQUIRE,
# experiment build), and the trace at depth 8 (more batches posted ahead).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 1
O=gpurun_out/r5h; mkdir -p $O; export TMPDIR=/tmp
AB=ccfd_demo_summit_amd/_native/ab
st() { echo "[r5h] $(date +%T) $*"; }
b() {   # b <name> <extra bench args> [env...]
  local n=$1 x=$2; shift 2
  st "$n"
  env "$@" timeout -k 10 240 python bench.py --model gbdt --steps 20 --warmup 5 $x > $O/$n.json 2> $O/$n.log \
    || { tail -30 $O/$n.log; exit 1; }
  python -c "import json; d=json.load(open('$O/$n.json')); print('$n', d['value'], d['p50_latency_us'], d['p99_latency_us'], d.get('precision_vs_fp32', {}).get('route_flips_outside_1e-2_band'), d.get('wire_stale_rows'), d['config'].get('depth'), d['config'].get('parallelism'))"
}
b default ""
b itrace --diagnostic CCFD_LIB_PATH=$AB/itrace.so CCFD_ITEM_TRACE_OUT=$O/itrace
python bench/experiments/item_trace.py $O/itrace.0 --json $O/itrace_phases.json
b itrace_d8 "--diagnostic --depth 8" CCFD_LIB_PATH=$AB/itrace.so CCFD_ITEM_TRACE_OUT=$O/itrace_d8
python bench/experiments/item_trace.py $O/itrace_d8.0 --json $O/itrace_d8_phases.json
b noacq_itrace --diagnostic CCFD_LIB_PATH=$AB/noacq_itrace.so CCFD_ITEM_TRACE_OUT=$O/noacq_itrace
python bench/experiments/item_trace.py $O/noacq_itrace.0 --json $O/noacq_itrace_phases.json
b noacq --diagnostic CCFD_LIB_PATH=$AB/noacq.so
b noacq_d8 "--diagnostic --depth 8" CCFD_LIB_PATH=$AB/noacq.so
b tkov --diagnostic CCFD_LIB_PATH=$AB/tkov.so
b default_again ""
st done
