#!/usr/bin/env bash
# Round-5 pass T (item 6): the persistent G20 path with the trees replaced by a use of the bins
# (CCFD_EXP_READ_ONLY): the same claims, zero-copy loads, outputs, release and tickets -- what
# the read + completion path sustains on its own, against the full kernel.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 1
O=gpurun_out/r5t; mkdir -p $O; export TMPDIR=/tmp
AB=ccfd_demo_summit_amd/_native/ab
st() { echo "[r5t] $(date +%T) $*"; }
b() {   # b <name> <extra args> [env...]
  local n=$1 x=$2; shift 2
  st "$n"
  env "$@" timeout -k 10 240 python bench.py --model gbdt --steps 20 --warmup 5 $x > $O/$n.json 2> $O/$n.log \
    || { tail -30 $O/$n.log; exit 1; }
  python -c "import json; d=json.load(open('$O/$n.json')); print('$n', d['value'], d['p50_latency_us'], d['p99_latency_us'], d['rows_scored'] == d['rows_expected'], d['h2d_zerocopy_ceiling_tx_s_rank0'])"
}
b default ""
b readonly "--diagnostic" CCFD_LIB_PATH=$AB/readonly.so
b readonly_g257 "--diagnostic --persist-grid 257" CCFD_LIB_PATH=$AB/readonly.so
b readonly_d8 "--diagnostic --depth 8" CCFD_LIB_PATH=$AB/readonly.so
st done
