set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python scripts/cluster_smoke.py --seconds 15 --count 2000000 --out gpurun_out/cluster_smoke.json > gpurun_out/cluster_smoke.log 2>&1 || { tail -20 gpurun_out/cluster_smoke.log; for f in gpurun_out/cluster/*.log; do echo "== $f"; tail -15 $f; done; exit 1; }
cat gpurun_out/cluster_smoke.json
