"""Config 4's persistent kernel alone, for ``rocprofv3 --pmc``.

Under counter collection rocprofv3 serialises dispatches: every kernel waits for the one
before it to end.  ``bench.py`` reads the device counters and all-reduces them (X2) while
the persistent kernel is resident, so under ``--pmc`` it deadlocks behind the kernel
(round-6 pass F, first attempt).  This driver issues no GPU work while the kernel is
resident: the model and the logs are set up first, the micro-batches go through the
engine's native pump (host doorbell ring, zero-copy rows and results), and closing the
engine ends the kernel -- the one dispatch whose counters the run collects.

    rocprofv3 --pmc SQ_WAVES ... --output-format csv -d out -o run -- \\
        python3 bench/pmc_persist.py --batches 20000

Prints one JSON line: rows, wall seconds, tx/s over the pumped region, and the fraud
hand-off totals (every fraud-routed row handed off).  Counter values per batch are
derived offline from the CSV (``scripts/pmc_table.py``).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="gbdt")
    ap.add_argument("--batches", type=int, default=20000)
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--depth", type=int, default=4)
    ap.add_argument("--streams", type=int, default=4)
    ap.add_argument("--partitions", type=int, default=2)     # bench.py: 2 partitions a rank
    ap.add_argument("--log-rows", type=int, default=1 << 22)
    ap.add_argument("--seed", type=int, default=0)
    a = ap.parse_args()
    import torch

    from ccfd_demo_summit_amd.data import FRAUD_RATE, generate
    from ccfd_demo_summit_amd.engine import PartitionLog, StreamEngine
    from ccfd_demo_summit_amd.models import build_model
    from ccfd_demo_summit_amd.parallel import broadcast_model, init_distributed
    from ccfd_demo_summit_amd.parallel.dp import resolve_row_format

    if not torch.cuda.is_available():
        raise SystemExit("pmc_persist.py needs a GPU")
    wire = resolve_row_format(a.model, "auto")
    ctx = init_distributed()
    Xcal, _ = generate(200_000, seed=a.seed + 999)
    model = build_model(a.model, seed=a.seed, X_ref=Xcal, calibrate_rate=FRAUD_RATE, threshold=0.5)
    dm = broadcast_model(ctx, model, a.model, wire)
    eng = StreamEngine(dm, batch=a.batch, depth=a.depth, streams=a.streams, input_mode="zerocopy", output_mode="zerocopy",
                       threshold=0.5, device=ctx.device.index, exec_mode="persistent", flag_capacity=1 << 23)
    rows_per_part = max(a.batch * 4, a.log_rows // a.partitions)
    logs = []
    for p in range(a.partitions):
        log = PartitionLog(rows_per_part, wire=dm.row_format == "w64", bins=dm.bins)
        Xp, _ = generate(rows_per_part, seed=a.seed * 7919 + p)
        log.write_rows(0, Xp)
        log.ids.array[:] = np.arange(rows_per_part, dtype=np.uint64) + np.uint64(p) * np.uint64(1 << 40)
        eng.add_log(p, log)
        logs.append(log)
    torch.cuda.synchronize()            # every setup dispatch done before the kernel is resident
    handed = [0]

    def handoff(records):
        handed[0] += len(records)

    t0 = time.perf_counter()
    st = eng.pump(a.batches, drain=True, on_flagged=handoff)
    dt = time.perf_counter() - t0
    handoff(eng.drain_flagged())
    eng.close()                         # the persistent kernel ends: its counters are collected
    print(json.dumps({"model": a.model, "row_format": dm.row_format, "batches": a.batches, "batch": a.batch,
                      "depth": a.depth, "rows": st.rows, "wall_s": round(dt, 4),
                      "tx_s": round(st.rows / max(dt, 1e-9), 1), "p50_us": round(st.lat_p50_us, 1),
                      "fraud_routed": st.fraud_rows, "handed_off": handed[0],
                      "lib": os.environ.get("CCFD_LIB_PATH", "default")}), flush=True)


if __name__ == "__main__":
    main()
