set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
R="$GRAFT_REPO_ROOT"
cd /tmp
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > "$R/gpurun_out/pmc_list.txt" 2>&1 || true
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES --output-format csv -d "$R/gpurun_out/pmc25a" -o run -- python3 "$R/bench.py" --steps 3 --warmup 1 --batches-per-step 64 --no-unloaded-probe > "$R/gpurun_out/pmc25a.log" 2>&1 || { tail -20 "$R/gpurun_out/pmc25a.log"; exit 1; }
ls "$R/gpurun_out/pmc25a"
