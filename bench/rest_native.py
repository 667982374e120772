#!/usr/bin/env python3
"""Seldon predict() REST throughput/latency through the native front end
(csrc/engine/seldon_http.cpp) with the native load generator (csrc/engine/http_load.cpp):
one transaction per request (the reference's batch=1 topology, README.md:549), N keep-alive
connections.  Scorer: the fused HIP kernel on the GPU (default) or CPU.

    python bench/rest_native.py [--model mlp] [--conns 1,16,64,256] [--seconds 5]
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="mlp", choices=["lr", "mlp", "gbdt"])
    ap.add_argument("--device", default="auto", choices=["auto", "gpu", "cpu"])
    ap.add_argument("--conns", default="1,16,64,256")
    ap.add_argument("--seconds", type=float, default=5.0)
    ap.add_argument("--rows-per-request", type=int, default=1)
    ap.add_argument("--workers", type=int, default=1, help="server epoll threads (one GPU engine each)")
    ap.add_argument("--client-threads", type=int, default=0, help="load generator threads (0 = 1 per 64 conns)")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    from ccfd_demo_summit_amd.contracts import seldon
    from ccfd_demo_summit_amd.data import FRAUD_RATE, generate
    from ccfd_demo_summit_amd.models import build_model
    from ccfd_demo_summit_amd.serving.native_seldon import NativeSeldonServer, http_load
    from ccfd_demo_summit_amd.serving.scorers import make_scorer
    X, _ = generate(100_000, seed=7)
    model = build_model(a.model, seed=0, X_ref=X, calibrate_rate=FRAUD_RATE)
    scorers = [make_scorer(model, 0.5, device=a.device, max_batch=4096) for _ in range(a.workers)]
    scorer = scorers[0]
    srv = NativeSeldonServer(scorers if a.workers > 1 else scorer, "127.0.0.1", 0, workers=a.workers)
    body = json.dumps(seldon.build_request(X[:a.rows_per_request])).encode()
    res = {"metric": "Seldon REST predict() through the native front end", "model": a.model,
           "scorer": getattr(scorer, "device", "cpu"), "rows_per_request": a.rows_per_request,
           "server_workers": a.workers, "runs": []}
    http_load("127.0.0.1", srv.port, body, conns=8, seconds=0.5)          # warm-up
    for c in [int(x) for x in a.conns.split(",")]:
        b0 = srv.stats()
        r = http_load("127.0.0.1", srv.port, body, conns=c, seconds=a.seconds, threads=a.client_threads)
        b1 = srv.stats()
        r.update(conns=c, tx_per_s=round(r["req_per_s"] * a.rows_per_request, 1),
                 mean_rows_per_gpu_call=round((b1["rows"] - b0["rows"]) / max(1, b1["batches"] - b0["batches"]), 2))
        r = {k: (round(v, 2) if isinstance(v, float) else v) for k, v in r.items()}
        res["runs"].append(r)
        print(json.dumps(r), flush=True)
    srv.stop()
    if a.out:
        Path(a.out).write_text(json.dumps(res, indent=1) + "\n")


if __name__ == "__main__":
    main()
