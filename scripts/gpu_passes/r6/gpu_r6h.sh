#!/usr/bin/env bash
# Round-6 pass H: the pump-only config-4 rate falls from 2.73e9 (1 s run) to 2.50-2.53e9 (5 s run,
# pass G).  Rate per 0.5 s segment, with and without fraud-routed rows (--fraud-rate 1e-7: almost none), and
# with a small flagged ring (drained often).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 1
O=gpurun_out/r6h; mkdir -p $O; export TMPDIR=/tmp PYTHONFAULTHANDLER=1
st() { echo "[r6h] $(date +%T) $*"; }
run() { n=$1; shift; st $n; timeout -k 10 180 python3 -u bench/pmc_persist.py --batches 200000 --segments 10 "$@" > $O/$n.json 2> $O/$n.log || { tail -20 $O/$n.log; exit 1; }; cat $O/$n.json; }
run default
run nofraud --fraud-rate 1e-7
run smallring --flag-capacity 1048576
run default_again
st done
