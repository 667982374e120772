set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof14_w64" -o run -- python3 "$R/bench.py" --steps 5 --warmup 2 --no-unloaded-probe --wire w64 > "$R/gpurun_out/prof14_w64.log" 2>&1 || { tail -20 "$R/gpurun_out/prof14_w64.log"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof14_f32" -o run -- python3 "$R/bench.py" --steps 5 --warmup 2 --no-unloaded-probe > "$R/gpurun_out/prof14_f32.log" 2>&1 || { tail -20 "$R/gpurun_out/prof14_f32.log"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof14_w64_b64k" -o run -- python3 "$R/bench.py" --steps 5 --warmup 2 --no-unloaded-probe --wire w64 --batch 65536 --batches-per-step 16 > "$R/gpurun_out/prof14_w64_b64k.log" 2>&1 || { tail -20 "$R/gpurun_out/prof14_w64_b64k.log"; exit 1; }
echo done
