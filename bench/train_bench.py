"""Trainer step rate on one GPU: eager vs HIP-graph-captured step (TrainConfig.graph).

    python bench/train_bench.py --rows 2000000 --batch 8192 --epochs 2
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from ccfd_demo_summit_amd.data import generate
from ccfd_demo_summit_amd.train import TrainConfig, evaluate, train_mlp


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=2_000_000)
    ap.add_argument("--batch", type=int, default=8192)
    ap.add_argument("--epochs", type=int, default=2)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    X, y = generate(a.rows, seed=1, fraud_rate=0.0172)
    Xv, yv = generate(50_000, seed=2, fraud_rate=0.0172)
    res = {}
    for graph in (False, True, False, True):           # second pair: warm caches / allocator
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        m, info = train_mlp(X, y, TrainConfig(epochs=a.epochs, batch=a.batch, device="cuda", graph=graph))
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        key = "graph" if graph else "eager"
        res[key] = {"steps": info["steps"], "seconds": round(dt, 3),
                    "steps_per_s": round(info["steps"] / dt, 1),
                    "samples_per_s": round(info["steps"] * a.batch / dt, 1),
                    "roc_auc": round(evaluate(m, Xv, yv)["roc_auc"], 4)}
    res["speedup"] = round(res["graph"]["steps_per_s"] / res["eager"]["steps_per_s"], 2)
    res["config"] = {"model": "mlp_30_128_64_1", "batch": a.batch, "rows": a.rows, "epochs": a.epochs,
                     "dtype": "bf16 autocast", "optimizer": "AdamW"}
    print(json.dumps(res), flush=True)
    if a.out:
        open(a.out, "w").write(json.dumps(res) + "\n")


if __name__ == "__main__":
    main()
