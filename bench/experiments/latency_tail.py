"""Where does the GBDT p99 tail come from?  Same engine (G32, persistent, depth 6,
65536-row batches), three pumping patterns: one long pump call; pump steps separated by
the bench's per-step host work (drain_flagged); pump steps separated by an idle gap.
Prints p50/p99 and the latency histogram's tail buckets for each."""
import json
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))


def main():
    from ccfd_demo_summit_amd.data import FRAUD_RATE, generate
    from ccfd_demo_summit_amd.engine import PartitionLog, StreamEngine
    from ccfd_demo_summit_amd.models import build_model
    from ccfd_demo_summit_amd.ops.kernels import DeviceModel
    from ccfd_demo_summit_amd.parallel import hist_quantile
    kind = sys.argv[1] if len(sys.argv) > 1 else "gbdt"
    B, depth = (65536, 6) if kind == "gbdt" else (4096, 16)
    Xc, _ = generate(200_000, seed=1)
    m = build_model(kind, seed=0, X_ref=Xc, calibrate_rate=FRAUD_RATE)
    dm = DeviceModel(m, "cuda", wire=kind != "gbdt", bins=True if kind == "gbdt" else None)
    logs = []
    eng = StreamEngine(dm, batch=B, depth=depth, streams=4, input_mode="zerocopy", exec_mode="persistent")
    for p in range(2):
        X, _ = generate(1 << 21, seed=p)
        log = PartitionLog.from_arrays(X, bins=dm.bins, wire=kind != "gbdt")
        eng.add_log(p, log)
        logs.append(log)
    eng.pump(200, drain=True)
    total = 20000 if kind == "gbdt" else 200000
    per = 410 if kind == "gbdt" else 3342

    def report(name, st, t):
        h = st.lat_hist.astype(np.int64)
        tail = {f"{2 ** (i / 4) / 1e3:.0f}us": int(h[i]) for i in range(256) if h[i] and 2 ** (i / 4) > 400e3}
        print(json.dumps({"pattern": name, "batches": int(st.batches), "tx_s": round(st.rows / t, 1),
                          "p50_us": round(hist_quantile(h, 0.5) / 1e3, 1), "p99_us": round(hist_quantile(h, 0.99) / 1e3, 1),
                          "p999_us": round(hist_quantile(h, 0.999) / 1e3, 1), "tail_buckets": tail}), flush=True)

    eng.reset_stats()
    t0 = time.perf_counter()
    eng.pump(total, drain=False)
    st = eng.pump(0, drain=True)
    report("one_pump_call", st, time.perf_counter() - t0)
    for name, gap in (("steps_drain_flagged", None), ("steps_idle_1ms", 1e-3), ("steps_poll_1ms", -1e-3),
                      ("steps_pyspin_1ms", "spin")):
        eng.reset_stats()
        t0 = time.perf_counter()
        rows = 0
        for _ in range(total // per):
            rows += eng.pump(per, drain=False).rows
            if gap is None:
                eng.drain_flagged()
            elif gap == "spin":                     # busy host thread, engine untouched
                t_end = time.perf_counter() + 1e-3
                while time.perf_counter() < t_end:
                    pass
            elif gap > 0:
                time.sleep(gap)
            else:                                   # busy gap: retire batches as they land
                t_end = time.perf_counter() - gap
                while time.perf_counter() < t_end:
                    eng.run(0, 0)
        st = eng.pump(0, drain=True)
        report(name, st, time.perf_counter() - t0)
    eng.close()


if __name__ == "__main__":
    main()
