"""Throughput-latency operating curve of the headline path on one GPU:
runs bench.py's measurement for each (depth, persistent grid, item rows) point in ONE
process and prints one JSON line per point (tx/s, p50, p99, device exec p50).

    python bench/operating_point.py --depths 8,12,16,24,32 --grids 128,256 --items 256,512
"""
from __future__ import annotations

import argparse
import itertools
import json
import os
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--depths", default="8,12,16,24,32")
    ap.add_argument("--grids", default="128")
    ap.add_argument("--items", default="512")
    ap.add_argument("--streams", default="4")
    ap.add_argument("--model", default="mlp")
    ap.add_argument("--log-rows", default=str(1 << 21), help="comma list: rows per rank")
    ap.add_argument("--steps", default="10", help="comma list")
    ap.add_argument("--extra", default="", help="extra bench.py args, ':'-separated")
    ap.add_argument("--envs", default="", help="'|'-separated env settings swept in-process, each "
                                               "'K=V+K2=V2' (kernel knobs read per launch, e.g. CCFD_G32_R)")
    ap.add_argument("--batches", default="", help="comma list of --batch values (default: bench's)")
    ap.add_argument("--exec-modes", default="auto", help="comma list of bench.py --exec-mode values")
    ap.add_argument("--min-timed-s", type=float, default=0.5)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    import bench
    rows = []
    grid_pts = itertools.product(args.exec_modes.split(","), args.envs.split("|"), (args.batches or "0").split(","),
                                 args.items.split(","),
                                 args.grids.split(","), args.depths.split(","), args.streams.split(","),
                                 args.log_rows.split(","), args.steps.split(","))
    for xmode, envset, batch, item, grid, depth, streams, lrows, steps in grid_pts:
        for kv in [e for e in envset.split("+") if e]:
            k, v = kv.split("=", 1)
            os.environ[k] = v
        os.environ["CCFD_PERSIST_ITEM_ROWS"] = item
        extra = [a for a in args.extra.split(":") if a] + (["--batch", batch] if batch != "0" else []) + \
            ["--exec-mode", xmode]
        with tempfile.NamedTemporaryFile("r", suffix=".json") as f:
            bench.main(["--model", args.model, "--steps", steps, "--warmup", "3", "--depth", depth,
                        "--persist-grid", grid, "--streams", streams,
                        "--min-timed-s", str(args.min_timed_s), "--log-rows", lrows,
                        "--precision-rows", "0", "--no-f32-probe", "--probe-ms", "0",
                        "--no-unloaded-probe", "--out", f.name] + extra)
            d = json.loads(Path(f.name).read_text())
        r = {"exec_mode": d["config"]["exec_mode"], "env": envset, "batch": int(batch), "item_rows": int(item), "grid": int(grid), "depth": int(depth),
             "streams": int(streams), "log_rows": int(lrows), "steps": int(steps),
             "tx_s": d["value"], "p50_us": d["p50_latency_us"], "p99_us": d["p99_latency_us"],
             "device_exec_us_p50": d["device_exec_us_p50"], "timed_s": d["timed_region_s"],
             "host_wait_us": d["host_us_per_batch"]["wait"], "exact": d["rows_scored"] == d["rows_expected"]}
        print("POINT " + json.dumps(r), flush=True)
        rows.append(r)
    if args.out:
        Path(args.out).write_text("\n".join(json.dumps(r) for r in rows) + "\n")


if __name__ == "__main__":
    main()
