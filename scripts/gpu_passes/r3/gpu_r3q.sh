#!/bin/bash
# Round-3 GPU pass Q: is the small-item cap the same-address counter atomics (16) or the
# output writes (32)?  Diagnostic ablations of the persistent kernels (timing only).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3q
mkdir -p $O
echo "[r3q] $(date +%T) pipelined items"
timeout -k 10 600 python bench/experiments/latency_breakdown.py --ablate 0,16,32,48 --pipe 1 --items 128 --grids 128,256 --depths 4,8,12 --batches 3000 --out $O/abl2_pipe.jsonl > $O/abl2_pipe.log 2>&1 || { tail -20 $O/abl2_pipe.log; exit 1; }
echo "[r3q] $(date +%T) claimed items"
timeout -k 10 600 python bench/experiments/latency_breakdown.py --ablate 0,16,32 --pipe 0 --items 512 --grids 64 --depths 8,12 --batches 3000 --out $O/abl2_claimed.jsonl > $O/abl2_claimed.log 2>&1 || { tail -20 $O/abl2_claimed.log; exit 1; }
python3 - <<'PY'
import json
for f in ("gpurun_out/r3q/abl2_pipe.jsonl", "gpurun_out/r3q/abl2_claimed.jsonl"):
    for l in open(f):
        d = json.loads(l)
        print(d["items"][:5], d["item_rows"], d["grid"], "abl", d["ablate"], "depth", d["depth"],
              "tx %.3g" % d["tx_s"], "p50", d["p50_total_us"], "dev", d["p50_dev_exec_us"])
PY
echo "[r3q] done"
