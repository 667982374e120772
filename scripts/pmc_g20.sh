#!/usr/bin/env bash
# Two rocprofv3 --pmc passes over the G20 GBDT launch kernel on 16M HBM-resident rows
# (profiles/r2/g20/pmc_gbdt_g20.txt).  gpurun -- 'bash scripts/pmc_g20.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/pmc_g20; mkdir -p $O
timeout -s KILL 90 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAVES SQ_WAVE_CYCLES --output-format csv -d $O/a -o run -- python3 bench/kernel_sol.py --cases gbdt/g20 --sizes 16777216 --iters 5 > $O/a.log 2>&1 || { tail -20 $O/a.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_WAIT_INST_ANY --output-format csv -d $O/b -o run -- python3 bench/kernel_sol.py --cases gbdt/g20 --sizes 16777216 --iters 5 > $O/b.log 2>&1 || { tail -20 $O/b.log; exit 1; }
find $O -name '*counter_collection.csv' | head
