#!/bin/bash
# Round-3 GPU pass I: where the unloaded micro-batch latency goes, by persistent item size
# and grid (the depth the link needs, hence p50 at full rate, follows from it).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3i
mkdir -p $O
step() { echo "[r3i] $(date +%T) $*"; }
step latency breakdown sweep
timeout -k 10 600 python bench/experiments/latency_breakdown.py --items 64,128,256,512 --grids 64,128,256 --depths 1,4,8,12 --batches 3000 --out $O/latency_sweep.jsonl > $O/latency_sweep.log 2>&1 || { tail -20 $O/latency_sweep.log; exit 1; }
cat $O/latency_sweep.jsonl
step kernel_sol default PF
timeout -k 10 300 python bench/kernel_sol.py --cases mlp:w64 --sizes 1048576,16777216 --tag quad_default > $O/sol_default.jsonl 2>$O/sol_default.err || { tail -20 $O/sol_default.err; exit 1; }
cat $O/sol_default.jsonl
step doorbell probe: host-memory vs fine-grained VRAM doorbell round trip
timeout -k 10 120 ./scripts/bin/doorbell_probe > $O/doorbell_probe.jsonl 2>&1 || { cat $O/doorbell_probe.jsonl; exit 1; }
cat $O/doorbell_probe.jsonl
step done
