#!/bin/bash
# Round-3 GPU pass H: four-tile epilogue of the W64 wire kernels (wire_body.h kQuad) --
# numerics, then HBM-resident speed-of-light with the old pair epilogue (PF=2) vs quad (PF=4).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3h
mkdir -p $O
step() { echo "[r3h] $(date +%T) $*"; }
step kernel numerics
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest_kernels.log 2>&1 || { tail -40 $O/pytest_kernels.log; exit 1; }
tail -3 $O/pytest_kernels.log
for pf in 2 4; do
  step kernel_sol MLP_PF=$pf
  CCFD_MLP_PF=$pf timeout -k 10 300 python bench/kernel_sol.py --cases mlp:w64,lr:w64 --sizes 1048576,16777216 --tag pf$pf > $O/sol_pf$pf.jsonl 2>$O/sol_pf$pf.err || { tail -20 $O/sol_pf$pf.err; exit 1; }
  cat $O/sol_pf$pf.jsonl
done
step latency breakdown of the persistent MLP W64 path
timeout -k 10 300 python bench/experiments/latency_breakdown.py --depths 1,2,4,8,12 --batches 4000 > $O/latency_breakdown.jsonl 2>$O/latency_breakdown.err || { tail -20 $O/latency_breakdown.err; exit 1; }
cat $O/latency_breakdown.jsonl
step done
