#!/usr/bin/env bash
# Round-6 pass G: why bench.py's config 4 (2.555e9) sits below the pump-only driver
# (bench/pmc_persist.py: 2.735e9 in pass F2).  A/B of the NUMA binding on both drivers.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 1
O=gpurun_out/r6g; mkdir -p $O; export TMPDIR=/tmp PYTHONFAULTHANDLER=1
st() { echo "[r6g] $(date +%T) $*"; }
st pump unbound
timeout -k 10 180 python3 -u bench/pmc_persist.py --batches 200000 > $O/pump_unbound.json 2> $O/pump_unbound.log || { tail -20 $O/pump_unbound.log; exit 1; }
cat $O/pump_unbound.json
st pump bound
timeout -k 10 180 python3 -u bench/pmc_persist.py --batches 200000 --numa-bind > $O/pump_bound.json 2> $O/pump_bound.log || { tail -20 $O/pump_bound.log; exit 1; }
cat $O/pump_bound.json
st bench bound
timeout -k 10 300 python3 -u bench.py --model gbdt --steps 20 --warmup 5 --out $O/bench_gbdt_bound.json > $O/bench_bound.log 2>&1 || { tail -30 $O/bench_bound.log; exit 1; }
tail -c 600 $O/bench_gbdt_bound.json; echo
st bench unbound
CCFD_NO_NUMA_BIND=1 timeout -k 10 300 python3 -u bench.py --model gbdt --steps 20 --warmup 5 --out $O/bench_gbdt_unbound.json > $O/bench_unbound.log 2>&1 || { tail -30 $O/bench_unbound.log; exit 1; }
tail -c 600 $O/bench_gbdt_unbound.json; echo
st done
