#!/usr/bin/env bash
# Round-6 pass F2: config 4's persistent G20 kernel under rocprofv3 --pmc, three builds:
#   default  -- the claimed kernel (the tree);
#   readonly -- the same protocol and row loads with the trees replaced by one use of the bins
#               (_native/ab/readonly.so, -D CCFD_EXP_READ_ONLY);
#   loader   -- the wave-specialised variant (1 loader wave, 2 LDS stages) as of commit 95a7cf0
#               (_native/ab/loader.so, built by scripts/build_ab.py --from-rev 95a7cf0; CCFD_G32_LOADER=1).
# bench.py deadlocks under --pmc (rocprofv3 serialises dispatches and bench reads counters while
# the kernel is resident), so the driver is bench/pmc_persist.py: no GPU work while the kernel runs.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../../.." && pwd)}"
O=$R/gpurun_out/r6f2; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
st() { echo "[r6f2] $(date +%T) $*"; }
N=40000
st plain default
timeout -k 10 180 python3 -u $R/bench/pmc_persist.py --batches $N > $O/plain_default.json 2> $O/plain_default.log \
  || { tail -20 $O/plain_default.log; exit 1; }
cat $O/plain_default.json
G1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SMEM"
G2="SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT"
G3="TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum GRBM_GUI_ACTIVE"
G4="SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM SQ_INST_LEVEL_LDS SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH"
for build in default readonly loader; do
  unset CCFD_LIB_PATH CCFD_G32_LOADER
  case $build in
    readonly) export CCFD_LIB_PATH=$R/ccfd_demo_summit_amd/_native/ab/readonly.so ;;
    loader)   export CCFD_LIB_PATH=$R/ccfd_demo_summit_amd/_native/ab/loader.so CCFD_G32_LOADER=1 ;;
  esac
  g=0
  for grp in "$G1" "$G2" "$G3" "$G4"; do
    g=$((g+1))
    st pmc $build group $g
    timeout -s KILL 150 rocprofv3 --pmc $grp --output-format csv -d $O/pmc_${build}_$g -o run -- \
      python3 -u $R/bench/pmc_persist.py --batches $N > $O/pmc_${build}_$g.json 2> $O/pmc_${build}_$g.log
    rc=$?
    tail -1 $O/pmc_${build}_$g.json
    if [ $rc -ne 0 ]; then
      tail -15 $O/pmc_${build}_$g.log
      # an unknown counter name fails fast (rc 1): go on; anything else (a kill, an abort) ends the pass
      [ $rc -eq 1 ] && grep -qi "counter" $O/pmc_${build}_$g.log || exit 1
    fi
  done
done
python3 $R/scripts/pmc_table.py $O > $O/pmc_table.md && cat $O/pmc_table.md
st done
