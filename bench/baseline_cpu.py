"""Config 1 of BASELINE.md, measured by us: the reference's scoring topology on CPU.

The reference scores every transaction with one synchronous REST call
(router -> Seldon ``POST /api/v0.1/predictions``, batch = 1, one model replica,
``SELDON_POOL_SIZE`` concurrent connections: deploy/model/modelfull.json:46,
deploy/router.yaml:63-68, README.md:549).  This script reproduces that topology with this
framework's own Seldon server (aiohttp, dynamic batching disabled: max_batch=1) serving a
30-feature logistic regression on the CPU, and ``pool`` concurrent async clients each posting one
transaction per request, for ``--seconds``.  The resulting tx/s is the denominator of
``vs_baseline`` in bench.py (key ``cpu_lr_batch1_seldon_rest_tx_per_s``).

    python bench/baseline_cpu.py --seconds 20 --pool 5 --write
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import socket
import subprocess
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

SERVER = r"""
import sys
sys.path.insert(0, {root!r})
from ccfd_demo_summit_amd.data import FRAUD_RATE, generate
from ccfd_demo_summit_amd.models import build_model
from ccfd_demo_summit_amd.serving.scorers import CpuScorer, GpuScorer
from ccfd_demo_summit_amd.serving.seldon_server import SeldonServer, run
X, _ = generate(50_000, seed=7)
m = build_model({model!r}, seed=0, X_ref=X, calibrate_rate=FRAUD_RATE)
scorer = GpuScorer(m, max_batch={max_batch}) if {gpu} else CpuScorer(m)
run(SeldonServer(scorer, max_batch={max_batch}, max_delay_us={delay}), host="127.0.0.1", port={port})
"""


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=15.0)
    ap.add_argument("--pool", type=int, default=5, help="SELDON_POOL_SIZE (reference default 5)")
    ap.add_argument("--write", action="store_true", help="write bench/baseline_measured.json")
    ap.add_argument("--scorer", default="cpu", choices=["cpu", "gpu"],
                    help="gpu: the same REST server with the fused HIP kernel + dynamic micro-batching")
    ap.add_argument("--model", default="lr", choices=["lr", "mlp"])
    ap.add_argument("--max-batch", type=int, default=1, help="server micro-batch cap (1 = reference batch=1)")
    ap.add_argument("--max-delay-us", type=int, default=0)
    ap.add_argument("--out", default=None)
    args = ap.parse_args(argv)

    import requests
    from ccfd_demo_summit_amd.contracts import seldon
    from ccfd_demo_summit_amd.data import generate

    port = _free_port()
    env = dict(os.environ)
    if args.scorer == "cpu":
        env.update(CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    code = SERVER.format(root=str(ROOT), port=port, model=args.model, gpu=args.scorer == "gpu",
                         max_batch=args.max_batch, delay=args.max_delay_us)
    srv = subprocess.Popen([sys.executable, "-c", code], env=env)
    url = f"http://127.0.0.1:{port}/api/v0.1/predictions"
    try:
        for _ in range(1800):
            try:
                if requests.get(f"http://127.0.0.1:{port}/health/ping", timeout=0.5).ok:
                    break
            except Exception:
                time.sleep(0.1)
        else:
            raise SystemExit("seldon server did not start")
        X, _ = generate(20_000, seed=3)
        bodies = [json.dumps(seldon.build_request(X[i:i + 1])) for i in range(len(X))]
        lat = [[] for _ in range(args.pool)]
        hdr = {"Content-Type": "application/json"}

        async def drive():
            import aiohttp
            conn = aiohttp.TCPConnector(limit=args.pool)
            async with aiohttp.ClientSession(connector=conn) as s:
                async def worker(k, stop):
                    i = k
                    while time.perf_counter() < stop:
                        t = time.perf_counter()
                        async with s.post(url, data=bodies[i % len(bodies)], headers=hdr) as r:
                            r.raise_for_status()
                            await r.read()
                        if stop != warm_stop:
                            lat[k].append(time.perf_counter() - t)
                        i += args.pool
                warm_stop = time.perf_counter() + 1.0      # warm connections + server
                await asyncio.gather(*(worker(k, warm_stop) for k in range(args.pool)))
                t0 = time.perf_counter()
                await asyncio.gather(*(worker(k, t0 + args.seconds) for k in range(args.pool)))
                return time.perf_counter() - t0

        wall = asyncio.run(drive())
        all_lat = np.concatenate([np.asarray(v) for v in lat]) * 1e6
        n = all_lat.size
        key = ("cpu_lr_batch1_seldon_rest_tx_per_s" if args.scorer == "cpu" and args.model == "lr"
               and args.max_batch == 1 else f"{args.scorer}_{args.model}_seldon_rest_tx_per_s")
        rec = {key: round(n / wall, 1),
               "p50_us": round(float(np.percentile(all_lat, 50)), 1),
               "p99_us": round(float(np.percentile(all_lat, 99)), 1),
               "requests": int(n), "seconds": args.seconds, "pool": args.pool, "wall_s": round(wall, 2),
               "model": args.model, "scorer": args.scorer, "max_batch": args.max_batch,
               "server": "aiohttp Seldon v0.1", "client": "aiohttp, pool concurrent batch-1 requests",
               "host_cpus": os.cpu_count(), "label": "measured by us (reference-topology equivalent)"}
        print(json.dumps(rec))
        if args.write:
            (ROOT / "bench" / "baseline_measured.json").write_text(json.dumps(rec, indent=1) + "\n")
        if args.out:
            Path(args.out).write_text(json.dumps(rec) + "\n")
        return rec
    finally:
        srv.terminate()
        try:
            srv.wait(10)
        except subprocess.TimeoutExpired:
            srv.kill()


if __name__ == "__main__":
    main()
