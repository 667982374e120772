"""Child process for test_persistent_queue_isolation: keep a persistent scoring kernel
resident (batches in flight, no drain) and check that work on fresh torch streams -- and on
the legacy default stream -- still completes.  A stream that the HIP runtime maps onto the
persistent kernel's hardware queue would sit behind the never-ending kernel.
Prints one line per stream and exits 0 when all complete, 3 on a stall."""
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import numpy as np
    import torch
    from ccfd_demo_summit_amd.data import generate
    from ccfd_demo_summit_amd.engine import PartitionLog, StreamEngine
    from ccfd_demo_summit_amd.models import build_model
    from ccfd_demo_summit_amd.ops.kernels import DeviceModel
    dev = torch.device("cuda", 0)
    X, _ = generate(1 << 16, seed=1)
    m = build_model("mlp", seed=0, X_ref=X, calibrate_rate=0.01)
    eng = StreamEngine(DeviceModel(m, dev, wire=True), batch=4096, depth=8, streams=4,
                       input_mode="zerocopy", exec_mode="persistent")
    log = PartitionLog.from_arrays(X, wire=True)
    eng.add_log(0, log)
    eng.pump(16, drain=False)                      # kernel resident from here on
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 12
    x = torch.ones(1 << 20, device=dev)
    stalled = []
    for i in range(n + 1):
        s = None if i == n else torch.cuda.Stream(dev, priority=(-1 if i % 3 == 2 else 0))
        done = threading.Event()

        def work():
            if s is None:
                y = (x * 2).sum().item()           # default stream + D2H copy
            else:
                with torch.cuda.stream(s):
                    y = (x * 2).sum()
                s.synchronize()
            done.set()
        t = threading.Thread(target=work, daemon=True)
        t0 = time.perf_counter()
        t.start()
        ok = done.wait(5.0)
        print(f"stream {i} {'default' if s is None else 'prio%d' % (-1 if i % 3 == 2 else 0)} "
              f"{'ok' if ok else 'STALLED'} {time.perf_counter() - t0:.3f}s", flush=True)
        if not ok:
            stalled.append(i)
            break
        eng.pump(4, drain=False)                   # keep batches flowing between probes
    if stalled:
        print("STALL", stalled, flush=True)
        os._exit(3)
    eng.pump(0, drain=True)
    eng.close()
    log.free()
    print("ALL_OK", flush=True)


if __name__ == "__main__":
    main()
