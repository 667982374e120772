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
    ap.add_argument("--threshold", type=float, default=0.5)
    ap.add_argument("--fraud-rate", type=float, default=None,
                    help="calibrated share of fraud-routed rows (default: the dataset prior, ~0.17 %%)")
    ap.add_argument("--segments", type=int, default=1,
                    help="pump --batches in this many equal segments, each one's rate reported "
                         "(the flagged ring is drained between segments)")
    ap.add_argument("--flag-capacity", type=int, default=1 << 23)
    ap.add_argument("--drainer", action="store_true",
                    help="hand off on a collector thread beside the pump (bench.py's way) instead of "
                         "draining between segments")
    ap.add_argument("--numa-bind", action="store_true", help="pin to the GPU's NUMA node first, as bench.py does")
    a = ap.parse_args()
    import torch

    from ccfd_demo_summit_amd.data import FRAUD_RATE, generate
    from ccfd_demo_summit_amd.engine import FlaggedDrainer, PartitionLog, StreamEngine
    from ccfd_demo_summit_amd.models import build_model
    from ccfd_demo_summit_amd.parallel import broadcast_model, init_distributed
    from ccfd_demo_summit_amd.parallel.dp import resolve_row_format

    if not torch.cuda.is_available():
        raise SystemExit("pmc_persist.py needs a GPU")
    wire = resolve_row_format(a.model, "auto")
    ctx = init_distributed()
    numa = None
    if a.numa_bind:
        from ccfd_demo_summit_amd.utils.numa import bind_to_gpu
        numa = bind_to_gpu(ctx.device.index)
    Xcal, _ = generate(200_000, seed=a.seed + 999)
    model = build_model(a.model, seed=a.seed, X_ref=Xcal, calibrate_rate=FRAUD_RATE if a.fraud_rate is None else a.fraud_rate,
                        threshold=a.threshold)
    dm = broadcast_model(ctx, model, a.model, wire)
    eng = StreamEngine(dm, batch=a.batch, depth=a.depth, streams=a.streams, input_mode="zerocopy", output_mode="zerocopy",
                       threshold=a.threshold, device=ctx.device.index, exec_mode="persistent",
                      flag_capacity=a.flag_capacity)
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

    mu = __import__("threading").Lock()

    def handoff(records):
        with mu:
            handed[0] += len(records)
    drainer = FlaggedDrainer(eng, handoff).start() if a.drainer else None

    seg_rates = []
    per = max(1, a.batches // max(1, a.segments))
    rows = fraud = 0
    t0 = time.perf_counter()
    for k in range(max(1, a.segments)):
        ts = time.perf_counter()
        st = eng.pump(per, drain=(k == a.segments - 1), on_flagged=handoff)
        if drainer is None:
            handoff(eng.drain_flagged())
        rows += st.rows
        fraud += st.fraud_rows
        seg_rates.append(round(st.rows / max(time.perf_counter() - ts, 1e-9) / 1e9, 4))
    if drainer is not None:
        drainer.stop()
    dt = time.perf_counter() - t0
    handoff(eng.drain_flagged())
    eng.close()                         # the persistent kernel ends: its counters are collected
    print(json.dumps({"model": a.model, "row_format": dm.row_format, "batches": a.batches, "batch": a.batch,
                      "depth": a.depth, "rows": rows, "wall_s": round(dt, 4),
                      "tx_s": round(rows / max(dt, 1e-9), 1), "segment_gtx_s": seg_rates,
                      "flag_full_events": st.flag_full_events, "p50_us": round(st.p50_us, 1),
                      "fraud_routed": fraud, "handed_off": handed[0],
                      "numa_node": numa, "lib": os.environ.get("CCFD_LIB_PATH", "default")}), flush=True)


if __name__ == "__main__":
    main()
