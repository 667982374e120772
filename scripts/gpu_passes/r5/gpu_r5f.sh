#!/usr/bin/env bash
# Round-5 pass F: where the persistent G20 kernel's time goes.  Config 4 on
# the default library, then three experiment builds of the same kernel (scripts/build_ab.py,
# loaded with CCFD_LIB_PATH, so the bench labels the lines diagnostic): the per-item phase
# trace (CCFD_EXP_ITEM_TRACE), an agent-scope instead of system-scope item release
# (CCFD_EXP_AGENT_RELEASE), no proba / route output stream (CCFD_EXP_NO_OUTPUTS), and the previous
# item's ticket taken beside the next claim (CCFD_EXP_TICKET_OVERLAP).  First: the back-pressure GPU
# test after the non-blocking epoch tick fix.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 1
O=gpurun_out/r5f; mkdir -p $O; export TMPDIR=/tmp
AB=ccfd_demo_summit_amd/_native/ab
st() { echo "[r5f] $(date +%T) $*"; }
b() {   # b <name> [env...]: one config-4 bench line
  local n=$1; shift
  st "$n"
  env "$@" timeout -k 10 240 python bench.py --model gbdt --steps 20 --warmup 5 $DIAG > $O/$n.json 2> $O/$n.log \
    || { tail -30 $O/$n.log; exit 1; }
  python -c "import json; d=json.load(open('$O/$n.json')); print('$n', d['value'], d['p50_latency_us'], d['p99_latency_us'], d.get('precision_vs_fp32', {}).get('route_flips_outside_1e-2_band'), d['config'].get('parallelism'))"
}
st bp_pytest
timeout -k 10 240 python -u -m pytest tests/test_engine_service_gpu.py -x -v --timeout 200 --timeout-method thread \
    -k back_pressure > $O/bp_pytest.log 2>&1; rc=$?
tail -3 $O/bp_pytest.log; [ $rc -ge 2 ] && exit $rc
DIAG= b gbdt_default
DIAG=--diagnostic
b gbdt_itrace CCFD_LIB_PATH=$AB/itrace.so CCFD_ITEM_TRACE_OUT=$O/itrace
python bench/experiments/item_trace.py $O/itrace.* --json $O/itrace_phases.json
b gbdt_tkov_itrace CCFD_LIB_PATH=$AB/tkov_itrace.so CCFD_ITEM_TRACE_OUT=$O/tkov_itrace
python bench/experiments/item_trace.py $O/tkov_itrace.* --json $O/tkov_itrace_phases.json
b gbdt_tkov CCFD_LIB_PATH=$AB/tkov.so
b gbdt_agentrel CCFD_LIB_PATH=$AB/agentrel.so
b gbdt_noout CCFD_LIB_PATH=$AB/noout.so
DIAG= b gbdt_default_again
st done
