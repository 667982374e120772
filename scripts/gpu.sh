#!/usr/bin/env bash
# One parameterised GPU-box runner (replaces the per-lease scripts of round 1).
#
#   gpurun --timeout 900 -- 'bash scripts/gpu.sh OUTDIR STEP [STEP ...]'
#
# Each STEP is one of
#   tests[:PYTEST_K]            pytest -m gpu (optionally -k PYTEST_K)
#   smoke                       __graft_entry__.smoke()
#   bench:NAME[:ARGS...]        python bench.py ARGS --out OUTDIR/bench_NAME.json
#   e2e:NAME[:ARGS...]          python bench/e2e.py ARGS --out OUTDIR/e2e_NAME.json
#   prof:NAME[:ARGS...]         rocprofv3 --kernel-trace --stats around bench.py ARGS
#   py:NAME:SCRIPT[:ARGS...]    python SCRIPT ARGS > OUTDIR/NAME.log
# ARGS inside a step are ':'-separated (no spaces), e.g. bench:gbdt:--model:gbdt:--batch:65536.
# Every GPU step runs under its own time limit; the first failing step ends the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O="gpurun_out/$1"; shift
mkdir -p "$O"
export TMPDIR=/tmp

fail() { echo "[gpu.sh] step '$1' failed (rc=$2)"; tail -40 "$3"; exit 1; }

for step in "$@"; do
  IFS=':' read -r -a F <<< "$step"
  kind=${F[0]}
  case "$kind" in
    tests)
      k=(); [ -n "${F[1]}" ] && k=(-k "${F[1]}")
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread "${k[@]}" \
        > "$O/pytest.log" 2>&1 || fail "$step" $? "$O/pytest.log"
      tail -1 "$O/pytest.log" ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 \
        || fail "$step" $? "$O/smoke.log"
      tail -1 "$O/smoke.log" ;;
    bench)
      name=${F[1]}
      timeout -k 10 300 python -u bench.py "${F[@]:2}" --out "$O/bench_$name.json" > "$O/bench_$name.log" 2>&1 \
        || fail "$step" $? "$O/bench_$name.log"
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], '%.4g tx/s' % d['value'], 'p50', d['p50_latency_us'], 'us, timed', d.get('timed_region_s'), 's')" \
        "$O/bench_$name.json" "$name" ;;
    e2e)
      name=${F[1]}
      timeout -k 10 200 python -u bench/e2e.py "${F[@]:2}" --out "$O/e2e_$name.json" > "$O/e2e_$name.log" 2>&1 \
        || fail "$step" $? "$O/e2e_$name.log"
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], '%.4g tx/s' % d['value'], 'p50', d.get('ring_arrival_to_scored_p50_us'))" \
        "$O/e2e_$name.json" "$name" ;;
    prof)
      name=${F[1]}
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_$name" -o run -- \
        python3 bench.py "${F[@]:2}" > "$O/prof_$name.log" 2>&1 || fail "$step" $? "$O/prof_$name.log"
      find "$O/prof_$name" -name '*kernel_stats.csv' -exec head -8 {} \; ;;
    py)
      name=${F[1]}; script=${F[2]}
      timeout -k 10 300 python -u "$script" "${F[@]:3}" > "$O/$name.log" 2>&1 || fail "$step" $? "$O/$name.log"
      tail -5 "$O/$name.log" ;;
    *) echo "[gpu.sh] unknown step '$step'"; exit 2 ;;
  esac
done
echo "[gpu.sh] all steps ok"
