"""Training job -- the batch analogue of the reference's JupyterHub + Spark workbench
(deploy/frauddetection_cr.yaml:7-53): train a fraud model on
``creditcard.csv`` (or synthetic rows of that shape), evaluate it on a held-out split and
save it as a versioned safetensors file that a running engine hot-swaps (``launch engine
--watch-model``).  Data-parallel under torchrun: DDP for LR/MLP, all-reduced histograms for
the GBDT (train/trainer.py); rank 0 evaluates and writes.

    python -m ccfd_demo_summit_amd.train --model mlp --out model.safetensors
    torchrun --nproc-per-node 2 -m ccfd_demo_summit_amd.train --model gbdt --csv creditcard.csv --out m.st
    python -m ccfd_demo_summit_amd.train --from-catboost model.json --out m.st   # import, no training
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np


def _serve_metrics(port: int):
    """TrainMetrics on :port/metrics in a daemon thread (stdlib HTTP server)."""
    import threading
    from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

    from ..metrics.exporter import CONTENT_TYPE, TrainMetrics
    tm = TrainMetrics()

    class H(BaseHTTPRequestHandler):
        def do_GET(self):
            body = tm.expose()
            self.send_response(200)
            self.send_header("Content-Type", CONTENT_TYPE)
            self.send_header("Content-Length", str(len(body)))
            self.end_headers()
            self.wfile.write(body)

        def log_message(self, *a):
            pass
    srv = ThreadingHTTPServer(("0.0.0.0", port), H)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    return tm


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--model", default="mlp", choices=["lr", "mlp", "gbdt"])
    ap.add_argument("--csv", default=None, help="creditcard.csv (Time, V1..V28, Amount, Class)")
    ap.add_argument("--rows", type=int, default=400_000, help="synthetic rows when no --csv")
    ap.add_argument("--fraud-rate", type=float, default=0.0017)
    ap.add_argument("--epochs", type=int, default=3)
    ap.add_argument("--batch", type=int, default=8192)
    ap.add_argument("--trees", type=int, default=100)
    ap.add_argument("--depth", type=int, default=6)
    ap.add_argument("--device", default="auto")
    ap.add_argument("--holdout", type=float, default=0.2)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--version", default="1")
    ap.add_argument("--out", required=True)
    ap.add_argument("--max-borders", type=int, default=31,
                    help="GBDT: split candidates per feature (<= 31 keeps every trained ensemble on the "
                         "20-byte G20 row format; <= 255 for G32)")
    ap.add_argument("--metrics-port", type=int, default=0,
                    help="serve the trainer's /metrics (the SparkMetrics dashboard series) on this port "
                         "(+ rank) while training; 0 = off")
    ap.add_argument("--from-catboost", default=None,
                    help="import an oblivious CatBoost JSON model (models/gbdt_import.py) instead of training")
    a = ap.parse_args(argv)
    if a.from_catboost:
        from ..models import save_model
        from ..models.gbdt_import import from_catboost_json
        m = from_catboost_json(a.from_catboost)
        save_model(m, a.out, version=a.version)
        print(json.dumps({"model": "gbdt", "imported": a.from_catboost, "out": a.out, "trees": m.n_trees,
                          "depth": m.depth}), flush=True)
        return 0

    import torch
    import torch.distributed as dist
    from ..data import generate
    from ..models import save_model
    from .trainer import TrainConfig, evaluate, train_logistic, train_mlp, train_oblivious_gbdt

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    tm = None
    if a.metrics_port:
        tm = _serve_metrics(a.metrics_port + int(os.environ.get("LOCAL_RANK", "0")))
        tm.workers.set(world)
    if world > 1 and not dist.is_initialized():
        use_gpu = a.device != "cpu" and torch.cuda.is_available()
        if use_gpu:
            torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
        dist.init_process_group("nccl" if use_gpu else "gloo")
    if a.csv:
        from ..data.csv_source import read_creditcard_csv
        X, y = read_creditcard_csv(a.csv)
        if y is None:
            raise SystemExit(f"{a.csv}: no Class column to train on")
    else:
        X, y = generate(a.rows, seed=a.seed, fraud_rate=a.fraud_rate)
    rng = np.random.default_rng(a.seed)
    idx = rng.permutation(len(X))
    n_test = int(len(X) * a.holdout)
    te, tr = idx[:n_test], idx[n_test:]
    dev = a.device
    if world > 1 and dev == "auto" and torch.cuda.is_available():
        dev = f"cuda:{torch.cuda.current_device()}"
    if a.model == "gbdt":
        model, info = train_oblivious_gbdt(X[tr], y[tr], n_trees=a.trees, depth=a.depth, device=dev,
                                           n_bins=a.max_borders + 1)
    else:
        cfg = TrainConfig(epochs=a.epochs, batch=a.batch, device=dev, seed=a.seed, metrics=tm)
        model, info = (train_mlp if a.model == "mlp" else train_logistic)(X[tr], y[tr], cfg)
    if rank == 0:
        metrics = evaluate(model, X[te], y[te]) if n_test and 0 < y[te].sum() < n_test else {}
        save_model(model, a.out, version=a.version)
        print(json.dumps({"model": a.model, "out": a.out, "world": world, "train": info, "holdout": metrics},
                         default=float), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
