#!/usr/bin/env bash
# Round-6 pass F: rocprofv3 evidence on the round-6 tree.
#  1. kernel trace + stats of config 2 (MLP, W64) and config 4 (GBDT, G20), as the driver runs them;
#  2. config 4's persistent G20 kernel under --pmc, the default build against the read-only
#     build (trees replaced by one use of the bins; CCFD_LIB_PATH=_native/ab/readonly.so): where
#     the gap between the link (read-only: ~97 % of it) and the full kernel (~89 %) goes.
#     One counter group per run (rocprofv3 does not split passes).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../../.." && pwd)}"
O=$R/gpurun_out/r6f; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
st() { echo "[r6f] $(date +%T) $*"; }
B="--steps 5 --warmup 2 --no-unloaded-probe --precision-rows 0 --no-f32-probe --encode-probe-rows 0"
st trace mlp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/mlp -o mlp -- python3 $R/bench.py --steps 5 --warmup 2 \
    > $O/bench_mlp.json 2> $O/mlp.log || { tail -30 $O/mlp.log; exit 1; }
st trace gbdt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/gbdt -o gbdt -- python3 $R/bench.py --model gbdt --steps 5 --warmup 2 \
    > $O/bench_gbdt.json 2> $O/gbdt.log || { tail -30 $O/gbdt.log; exit 1; }
find $O -name "*.db" -size +20M -delete
G1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SMEM"
G2="SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT"
G3="TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum"
for build in default readonly; do
  if [ $build = readonly ]; then export CCFD_LIB_PATH=$R/ccfd_demo_summit_amd/_native/ab/readonly.so; else unset CCFD_LIB_PATH; fi
  g=0
  for grp in "$G1" "$G2" "$G3"; do
    g=$((g+1))
    st pmc $build group $g
    timeout -s KILL 240 rocprofv3 --pmc $grp --output-format csv -d $O/pmc_${build}_$g -o run -- \
      python3 $R/bench.py --model gbdt $B --diagnostic > $O/pmc_${build}_$g.json 2> $O/pmc_${build}_$g.log \
      || { tail -20 $O/pmc_${build}_$g.log; exit 1; }
  done
done
find $O -name "*counter_collection.csv" | head -20
st done
