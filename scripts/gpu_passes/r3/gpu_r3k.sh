#!/bin/bash
# Round-3 GPU pass K: pipelined static persistent items -- exactness, latency sweep, bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3k
mkdir -p $O
step() { echo "[r3k] $(date +%T) $*"; }
step pipe-item tests
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py tests/test_rules_gpu.py -x -q --timeout 120 --timeout-method thread -k "pipe or persistent" > $O/pytest_pipe.log 2>&1 || { tail -40 $O/pytest_pipe.log; exit 1; }
tail -3 $O/pytest_pipe.log
step latency sweep pipelined items
timeout -k 10 600 python bench/experiments/latency_breakdown.py --pipe 1 --items 64,128 --grids 64,128,256 --depths 1,2,4,6,8,12 --batches 3000 --out $O/pipe_sweep.jsonl > $O/pipe_sweep.log 2>&1 || { tail -20 $O/pipe_sweep.log; exit 1; }
cat $O/pipe_sweep.jsonl
step done
