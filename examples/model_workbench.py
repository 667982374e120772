"""Fraud-model workbench: the interactive model-development loop of the reference's
JupyterHub + Spark workbench (deploy/frauddetection_cr.yaml:7-53),
as a script to run, or to paste into a notebook cell by cell (the ``# %%`` markers).

1. load ``creditcard.csv`` (Time, V1..V28, Amount, Class), or synthetic rows of its shape;
2. train the three model families the engine serves (LR, MLP, oblivious GBDT);
3. compare them on a held-out split (ROC-AUC, PR-AUC);
4. check that the GBDT's exact 32-byte G32 wire picks the f32 model's leaves;
5. save versioned safetensors files a running engine hot-swaps (``launch engine --watch-model``);
6. with an MI355X visible, score through the HIP kernels and compare with the CPU models.

    python examples/model_workbench.py [--csv creditcard.csv] [--rows 200000] [--out models_out]

Multi-GPU training is the batch job: ``torchrun --nproc-per-node N -m ccfd_demo_summit_amd.train``.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main(argv=None) -> dict:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--csv", default="")
    ap.add_argument("--rows", type=int, default=200_000)
    ap.add_argument("--trees", type=int, default=100)
    ap.add_argument("--epochs", type=int, default=3)
    ap.add_argument("--batch", type=int, default=8192)
    ap.add_argument("--device", default="auto", help="auto | cpu | cuda:N")
    ap.add_argument("--out", default="models_out")
    a = ap.parse_args(argv)

    # %% data
    import numpy as np
    import torch

    from ccfd_demo_summit_amd.data import generate
    from ccfd_demo_summit_amd.models import load_model, save_model
    from ccfd_demo_summit_amd.train.trainer import (TrainConfig, evaluate, train_logistic, train_mlp,
                                                    train_oblivious_gbdt)
    if a.csv:
        from ccfd_demo_summit_amd.data.csv_source import read_creditcard_csv
        X, y = read_creditcard_csv(a.csv)
        if y is None:
            raise SystemExit(f"{a.csv}: no Class column")
    else:
        X, y = generate(a.rows, seed=0, fraud_rate=0.0017)
    idx = np.random.default_rng(0).permutation(len(X))
    n_test = len(X) // 5
    Xte, yte, Xtr, ytr = X[idx[:n_test]], y[idx[:n_test]], X[idx[n_test:]], y[idx[n_test:]]
    device = a.device if a.device != "auto" else ("cuda:0" if torch.cuda.is_available() else "cpu")
    print(f"{len(X)} rows, {int(y.sum())} fraud ({y.mean():.4%}), training on {device}")

    # %% train the three model families
    cfg = TrainConfig(epochs=a.epochs, batch=a.batch, device=device)
    models = {"lr": train_logistic(Xtr, ytr, cfg)[0], "mlp": train_mlp(Xtr, ytr, cfg)[0],
              "gbdt": train_oblivious_gbdt(Xtr, ytr, n_trees=a.trees, depth=6, device=device)[0]}
    report = {"rows": int(len(X)), "device": device, "models": {}}
    for name, m in models.items():
        r = evaluate(m, Xte, yte)
        report["models"][name] = r
        print(f"{name:5s} ROC-AUC {r['roc_auc']:.4f}  PR-AUC {r['pr_auc']:.4f}")

    # %% G32: one u8 bin per feature against the ensemble's own split thresholds
    gb = models["gbdt"]
    spec = gb.bin_spec()
    rows = spec.encode(Xte)
    same = bool(np.array_equal(gb.leaf_index(Xte), gb.leaf_index_g32(rows, spec)))
    report["g32"] = {"rows": int(len(rows)), "leaves_equal": same, "stamp": int(spec.stamp),
                     "edges": int(spec.offsets[-1])}
    print(f"G32: {len(rows)} rows, leaves identical to f32: {same}, {int(spec.offsets[-1])} edges, stamp {spec.stamp}")
    if not same:
        raise SystemExit("G32 leaves differ from the f32 model's")

    # %% save versioned models for the engine's hot swap
    os.makedirs(a.out, exist_ok=True)
    for name, m in models.items():
        path = os.path.join(a.out, f"{name}.safetensors")
        save_model(m, path, version="1")
        back = load_model(path)
        assert np.allclose(back.predict_proba(Xte[:1000]), m.predict_proba(Xte[:1000]), atol=1e-6)
        print("saved", path)

    # %% score through the MI355X kernels
    if torch.cuda.is_available() and device.startswith("cuda"):
        from ccfd_demo_summit_amd.engine import StreamEngine
        from ccfd_demo_summit_amd.ops.kernels import DeviceModel
        report["gpu"] = {}
        n = min(len(Xte), 100_000)
        for name, m in models.items():
            eng = StreamEngine(DeviceModel(m, torch.device(device), bins=(name == "gbdt")), batch=4096, depth=4)
            try:
                p, route = eng.score(Xte[:n])
            finally:
                eng.close()
            err = float(np.abs(p - m.predict_proba(Xte[:n])).max())
            report["gpu"][name] = {"max_abs_dp": err, "fraud_routed": int(route.sum())}
            print(f"{name:5s} GPU max |dp| {err:.2e}, {int(route.sum())} rows routed to the fraud process")
    print(json.dumps(report))
    return report


if __name__ == "__main__":
    main()
