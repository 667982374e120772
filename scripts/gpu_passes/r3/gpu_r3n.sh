#!/bin/bash
# Round-3 GPU pass N: LDS-staged flag lists in the W64 streaming bodies -- numerics, kernel SOL,
# then the 8-rank bench rehearsal on one GPU (gloo) for the N = 8 code paths.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3n
mkdir -p $O
step() { echo "[r3n] $(date +%T) $*"; }
step kernel + engine numerics
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py tests/test_rules_gpu.py -x -q --timeout 180 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
step kernel_sol
timeout -k 10 300 python bench/kernel_sol.py --cases mlp:w64,lr:w64 --sizes 1048576,16777216 --tag flagstage > $O/sol.jsonl 2>$O/sol.err || { tail -20 $O/sol.err; exit 1; }
cat $O/sol.jsonl
step 8-rank bench rehearsal
timeout -k 10 600 bash scripts/rehearse_dp.sh r3n/dp8 8 --steps 20 --warmup 5 > $O/rehearse8.log 2>&1 || { tail -40 $O/rehearse8.log; exit 1; }
tail -5 $O/rehearse8.log
step done
