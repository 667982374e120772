"""Sweep engine knobs (input/output mode, depth, streams, batch) on one GPU in ONE process
(interleaved rounds, cdna_hip_programming.md §5.4 rule 24) and print tx/s + latency.

    python bench/engine_sweep.py --rounds 3 --batches 512
"""
from __future__ import annotations

import argparse
import itertools
import json
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--batches", type=int, default=512)
    ap.add_argument("--log-rows", type=int, default=1 << 22)
    ap.add_argument("--model", default="mlp")
    ap.add_argument("--modes", default="dma:zerocopy,zerocopy:zerocopy,dma:dma")
    ap.add_argument("--depths", default="4,8,16")
    ap.add_argument("--streams", default="1,2,4")
    ap.add_argument("--batch-sizes", default="4096")
    args = ap.parse_args()

    import torch
    from ccfd_demo_summit_amd.data import generate
    from ccfd_demo_summit_amd.engine import PartitionLog, StreamEngine
    from ccfd_demo_summit_amd.models import build_model
    from ccfd_demo_summit_amd.ops.kernels import DeviceModel

    dev = torch.device("cuda", 0)
    Xc, _ = generate(100_000, seed=1)
    m = build_model(args.model, seed=0, X_ref=Xc, calibrate_rate=0.00172)
    dm = DeviceModel(m, dev)
    log = PartitionLog(args.log_rows)
    generate(args.log_rows, seed=3, out=log.feats.array)
    log.ids.array[:] = np.arange(args.log_rows, dtype=np.uint64)
    combos = list(itertools.product(args.modes.split(","), [int(d) for d in args.depths.split(",")],
                                    [int(s) for s in args.streams.split(",")],
                                    [int(b) for b in args.batch_sizes.split(",")]))
    engines = {}
    for mode, depth, streams, bs in combos:
        im, om = mode.split(":")
        e = StreamEngine(dm, batch=bs, depth=depth, streams=streams, input_mode=im, output_mode=om)
        e.add_log(0, log)
        e.pump(64, drain=True)
        engines[(mode, depth, streams, bs)] = e
    res = {k: [] for k in engines}
    for r in range(args.rounds):
        for k, e in engines.items():
            e.reset_stats()
            e.drain_flagged()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            st = e.pump(args.batches, drain=True)
            dt = time.perf_counter() - t0
            e.drain_flagged()
            nb = max(1, st.batches)
            res[k].append((st.rows / dt, st.p50_us, st.p99_us, st.host_submit_s / nb * 1e6,
                           st.host_wait_s / nb * 1e6, st.host_complete_s / nb * 1e6, dt / nb * 1e6))
    for k, v in res.items():
        tx = sorted(x[0] for x in v)
        print(json.dumps({"mode": k[0], "depth": k[1], "streams": k[2], "batch": k[3],
                          "tx_per_s_median": round(tx[len(tx) // 2] / 1e6, 2), "tx_per_s_max": round(tx[-1] / 1e6, 2),
                          "p50_us": round(v[-1][1], 1), "p99_us": round(v[-1][2], 1),
                          "us_per_batch": round(v[-1][6], 2), "host_submit_us": round(v[-1][3], 2),
                          "host_wait_us": round(v[-1][4], 2), "host_complete_us": round(v[-1][5], 2)}), flush=True)
    for e in engines.values():
        e.close()
    log.free()


if __name__ == "__main__":
    main()
