#!/bin/bash
# Round-3 GPU pass J: wave-level persistent work items -- exactness first, then the latency /
# throughput sweep against the workgroup items, then the bench with the best point.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3j
mkdir -p $O
step() { echo "[r3j] $(date +%T) $*"; }
step wave-item tests
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py tests/test_rules_gpu.py -x -q --timeout 120 --timeout-method thread -k "wave or persistent" > $O/pytest_wave.log 2>&1 || { tail -40 $O/pytest_wave.log; exit 1; }
tail -3 $O/pytest_wave.log
step latency sweep wave items
timeout -k 10 600 python bench/experiments/latency_breakdown.py --wave-tiles 4,8,16 --grids 64,128,256 --depths 1,4,6,8,12 --batches 3000 --out $O/wave_sweep.jsonl > $O/wave_sweep.log 2>&1 || { tail -20 $O/wave_sweep.log; exit 1; }
cat $O/wave_sweep.jsonl
step done
