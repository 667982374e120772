#!/usr/bin/env bash
# G20 persistent-kernel operating-point sweep on one MI355X (profiles/r2/g20/):
#   bash scripts/g20_sweep.sh OUTDIR "GRIDS" "ITEM_ROWS" "DEPTHS" [INFLIGHT]
# at BASELINE config 4 (100 x 6 oblivious GBDT, 65536-row micro-batches).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-g20c}; mkdir -p "$O"
for g in ${2:-128 192 256}; do
  for it in ${3:-512 1024}; do
    for d in ${4:-3 4}; do
      n=b_g${g}_i${it}_d${d}_f${5:-0}
      CCFD_G32_INFLIGHT=${5:-0} CCFD_PERSIST_ITEM_ROWS=$it timeout -k 10 200 python -u bench.py --model gbdt \
        --depth "$d" --persist-grid "$g" --no-unloaded-probe --precision-rows 0 --no-f32-probe \
        --out "$O/$n.json" > "$O/$n.log" 2>&1 || exit 1
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], '%.4g'%d['value'], d['p50_latency_us'], d['p99_latency_us'], d['device_exec_us_p50'])" "$O/$n.json" "$n" | tee -a "$O/sweep.txt"
    done
  done
done
