#!/usr/bin/env bash
# Soak run of the end-to-end loop (bench/e2e.py) with a resource sampler: every 5 s one CSV
# line of elapsed seconds, the e2e process tree's RSS (MiB) and the GPU's used VRAM (MiB), so
# a leak in the host runtime, the rings or the device allocations shows as a trend.
#   bash scripts/soak.sh OUTDIR SECONDS [e2e args ...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O="gpurun_out/$1"; S=$2; shift 2
mkdir -p "$O"
timeout -k 10 $((S + 120)) python -u bench/e2e.py --seconds "$S" --out "$O/e2e_soak.json" "$@" > "$O/e2e_soak.log" 2>&1 &
pid=$!
echo "t_s,rss_mib,vram_mib" > "$O/resources.csv"
t0=$(date +%s)
tree_rss() {   # RSS of $1 and its descendants, MiB
  local pids="$1" all="$1" kids
  while [ -n "$pids" ]; do
    kids=$(for p in $pids; do cat /proc/$p/task/*/children 2>/dev/null; done | tr '\n' ' ')
    all="$all $kids"; pids="$kids"
  done
  for p in $all; do awk '/VmRSS/ {print $2}' /proc/$p/status 2>/dev/null; done | awk '{s+=$1} END {printf "%.1f", s/1024}'
}
vram() { rocm-smi --showmeminfo vram --csv 2>/dev/null | awk -F, 'NR==2 {printf "%.1f", $3/1048576}'; }
while kill -0 $pid 2>/dev/null; do
  echo "$(( $(date +%s) - t0 )),$(tree_rss $pid),$(vram)" >> "$O/resources.csv"
  sleep 5
done
wait $pid; rc=$?
tail -3 "$O/resources.csv"
[ $rc -eq 0 ] || { echo "[soak] e2e exited rc=$rc"; tail -30 "$O/e2e_soak.log"; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('soak %.0f s' % d['seconds'], '%.4g tx/s' % d['value'], 'p50', d['ring_arrival_to_scored_p50_us'], 'p99', d['ring_arrival_to_scored_p99_us'])" "$O/e2e_soak.json"
