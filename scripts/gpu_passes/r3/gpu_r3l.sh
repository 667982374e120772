#!/bin/bash
# Round-3 GPU pass L: what the per-item fences cost (diagnostic ablations; outputs of ablated
# runs are not trusted, only their timing), claimed 512-row vs pipelined 64/128-row items.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3l
mkdir -p $O
step() { echo "[r3l] $(date +%T) $*"; }
step ablation sweep pipelined
timeout -k 10 600 python bench/experiments/latency_breakdown.py --ablate 0,64,512,576 --pipe 1 --items 64,128 --grids 128 --depths 1,4,8,12 --batches 3000 --out $O/abl_pipe.jsonl > $O/abl_pipe.log 2>&1 || { tail -20 $O/abl_pipe.log; exit 1; }
cat $O/abl_pipe.jsonl
step ablation sweep claimed 512
timeout -k 10 600 python bench/experiments/latency_breakdown.py --ablate 0,64,512,576 --pipe 0 --items 512 --grids 64 --depths 1,4,8,12 --batches 3000 --out $O/abl_claimed.jsonl > $O/abl_claimed.log 2>&1 || { tail -20 $O/abl_claimed.log; exit 1; }
cat $O/abl_claimed.jsonl
step done
