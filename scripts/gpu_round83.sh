set -o pipefail
cd "$GRAFT_REPO_ROOT"
R="$GRAFT_REPO_ROOT"
O=$R/gpurun_out/r83; mkdir -p $O
cd /tmp
export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --output-format csv -d $O/pmc1 -o run -- python3 $R/bench/kernel_sol.py --cases mlp:w64 --sizes 16777216 --iters 2 > $O/pmc1.log 2>&1 || { tail -20 $O/pmc1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_INSTS_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_LDS --output-format csv -d $O/pmc2 -o run -- python3 $R/bench/kernel_sol.py --cases mlp:w64 --sizes 16777216 --iters 2 > $O/pmc2.log 2>&1 || { tail -20 $O/pmc2.log; exit 1; }
find $O -name "*counter_collection.csv" | sort
