#!/usr/bin/env python3
"""Where does a micro-batch's latency go?  The headline's second number is p50 latency
(BASELINE.json metric), and by Little's law p50 = batches in flight / batch rate: the depth the
link needs to stay busy is set by the *unloaded* latency of one batch.  This traces every batch
(engine trace: host submit, device start / end on the device wall clock, host landed) at
several depths of the persistent MLP W64 path and splits the latency into

* dev_exec  : device start (chunk 0 claimed, descriptor read) -> last chunk's ticket;
* outside   : total - dev_exec = host post -> device start + device end -> host sees the
              completion record (the device/host clock offset cancels in the sum);

and, with the device/host offset pinned by the fastest depth-1 batch (an upper bound on
the offset, so `post_to_start` is a lower bound), post -> start and end -> landed separately.

    python bench/experiments/latency_breakdown.py [--depths 1,2,4,8,12] [--batches 4000]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))


def pct(a, q):
    return round(float(np.percentile(a, q)), 2) if len(a) else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--depths", default="1,2,4,8,12")
    ap.add_argument("--batches", type=int, default=4000)
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--grids", default="0", help="comma list of persistent grids (0 = engine default)")
    ap.add_argument("--items", default="0", help="comma list of CCFD_PERSIST_ITEM_ROWS (0 = engine default)")
    ap.add_argument("--pipe", default="0", help="comma list of CCFD_PERSIST_PIPE values (1 = pipelined "
                                               "static items, 0 = claimed workgroup items)")
    ap.add_argument("--log-rows", type=int, default=1 << 21)
    ap.add_argument("--tag", default="")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import torch
    from ccfd_demo_summit_amd.data import generate
    from ccfd_demo_summit_amd.engine import PartitionLog, StreamEngine
    from ccfd_demo_summit_amd.models import build_model
    from ccfd_demo_summit_amd.ops.kernels import DeviceModel

    dev = torch.device("cuda", 0)
    X, _ = generate(200_000, seed=1)
    m = build_model("mlp", seed=0, X_ref=X, calibrate_rate=0.00172)
    dm = DeviceModel(m, dev, wire=True)
    log = PartitionLog(a.log_rows, wire=True)
    Xl, _ = generate(a.log_rows, seed=2)
    log.write_rows(0, Xl)
    del Xl
    out = []
    pts = [(int(w), int(i), int(gr), int(d)) for w in a.pipe.split(",")
           for i in a.items.split(",") for gr in a.grids.split(",") for d in a.depths.split(",")]
    for pipe, item, grid, depth in pts:
        os.environ["CCFD_PERSIST_PIPE"] = str(pipe)
        if item:
            os.environ["CCFD_PERSIST_ITEM_ROWS"] = str(item)
        else:
            os.environ.pop("CCFD_PERSIST_ITEM_ROWS", None)
        eng = StreamEngine(dm, batch=a.batch, depth=depth, streams=1, input_mode="zerocopy",
                           output_mode="zerocopy", device=0, exec_mode="persistent",
                           persist_grid=grid)
        eng.add_log(0, log)
        eng.pump(500, drain=True)                      # warm: kernel resident, pages touched
        eng.reset_stats()
        eng.enable_trace(a.batches + 64)
        st = eng.pump(a.batches, drain=True)
        tr = eng.read_trace()
        eng.close()
        tr = tr[tr["t_landed"] > 0]
        total = (tr["t_landed"] - tr["t_submit"]) / 1e3
        dev_ok = tr["dev_end"] > tr["dev_start"]
        dexec = (tr["dev_end"] - tr["dev_start"])[dev_ok] / 1e3
        outside = total[dev_ok] - dexec
        # device/host clock offset: dev_start - t_submit >= offset; the fastest batch bounds it
        d0 = (tr["dev_start"] - tr["t_submit"])[dev_ok]
        off = float(d0.min())
        post_to_start = (d0 - off) / 1e3
        end_to_landed = (tr["t_landed"][dev_ok] - tr["dev_end"][dev_ok] + off) / 1e3
        pickup = (tr["t_complete"] - tr["t_landed"]) / 1e3
        r = {"tag": a.tag, "depth": depth, "batch": a.batch, "batches": int(len(tr)),
             "tx_s": round(st.rows / st.wall_s, 1) if st.wall_s else None,
             "p50_total_us": pct(total, 50), "p99_total_us": pct(total, 99),
             "p50_dev_exec_us": pct(dexec, 50), "p50_outside_us": pct(outside, 50),
             "min_outside_us": round(float(outside.min()), 2) if len(outside) else None,
             "p50_post_to_start_us_rel": pct(post_to_start, 50),
             "p50_end_to_landed_us_rel": pct(end_to_landed, 50),
             "p50_host_pickup_us": pct(pickup, 50),
             "grid": grid or "default", "item_rows": item or "default",
             "items": "pipelined-static" if pipe else "claimed"}
        print(json.dumps(r), flush=True)
        out.append(r)
    if a.out:
        Path(a.out).write_text("\n".join(json.dumps(r) for r in out) + "\n")


if __name__ == "__main__":
    main()
