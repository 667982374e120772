"""Trainers (LR / MLP / oblivious GBDT) learn the synthetic fraud signal and export into the
kernel model containers; tracing spans export valid Chrome-trace JSON."""
import json

import numpy as np
import pytest

from ccfd_demo_summit_amd.data import generate
from ccfd_demo_summit_amd.models import MLPModel, ObliviousGBDT
from ccfd_demo_summit_amd.models.mlp import emulate_packed_kernel
from ccfd_demo_summit_amd.train import TrainConfig, evaluate, train_logistic, train_mlp, train_oblivious_gbdt
from ccfd_demo_summit_amd.utils.tracing import Tracer


@pytest.fixture(scope="module")
def data():
    X, y = generate(40_000, seed=1, fraud_rate=0.02)
    Xv, yv = generate(10_000, seed=2, fraud_rate=0.02)
    return X, y, Xv, yv


def test_train_logistic(data):
    X, y, Xv, yv = data
    m, info = train_logistic(X, y, TrainConfig(epochs=3, lr=3e-2, device="cpu"))
    assert evaluate(m, Xv, yv)["roc_auc"] > 0.9
    assert len(m.pack()) == 448


def test_train_mlp_exports_packable_model(data):
    X, y, Xv, yv = data
    m, info = train_mlp(X, y, TrainConfig(epochs=2, device="cpu"))
    assert isinstance(m, MLPModel) and info["steps"] > 0
    assert evaluate(m, Xv, yv)["roc_auc"] > 0.9
    # the trained weights go through the same packing the HIP kernel consumes
    np.testing.assert_allclose(emulate_packed_kernel(m.pack(), Xv[:20]),
                               m.predict_proba(Xv[:20], emulate_bf16=True), atol=1e-6)


def test_train_oblivious_gbdt(data):
    X, y, Xv, yv = data
    g, info = train_oblivious_gbdt(X, y, n_trees=15, depth=4, device="cpu")
    assert isinstance(g, ObliviousGBDT) and g.feat.shape == (15, 4)
    assert evaluate(g, Xv, yv)["roc_auc"] > 0.9
    assert ObliviousGBDT.unpack(g.pack()).leaves.shape == (15, 16)


def test_tracer_chrome_json(tmp_path):
    t = Tracer(enabled=True, roctx=False)
    with t.span("pump", batches=3):
        with t.span("kernel"):
            pass
    t.instant("flip")
    t.counter("rows", value=5)
    p = t.dump(str(tmp_path / "trace.json"))
    doc = json.load(open(p))
    names = [e["name"] for e in doc["traceEvents"]]
    assert names.count("pump") == 1 and "kernel" in names and "flip" in names
    assert all("ts" in e for e in doc["traceEvents"])
    off = Tracer(enabled=False)
    with off.span("x"):
        pass
    assert off.events() == []
