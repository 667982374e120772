"""Trainer on the GPU: the HIP-graph-captured step (TrainConfig.graph) learns as well as the
eager step, for the bf16 MLP and the fp32 LR."""
import pytest
import torch

from ccfd_demo_summit_amd.data import generate
from ccfd_demo_summit_amd.train import TrainConfig, evaluate, train_logistic, train_mlp

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def data():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    X, y = generate(60_000, seed=1, fraud_rate=0.02)
    Xv, yv = generate(10_000, seed=2, fraud_rate=0.02)
    return X, y, Xv, yv


@pytest.mark.parametrize("graph", [True, False])
def test_train_mlp_gpu(data, graph):
    X, y, Xv, yv = data
    m, info = train_mlp(X, y, TrainConfig(epochs=3, batch=4096, device="cuda", graph=graph))
    assert bool(info.get("graph", False)) == graph
    assert info["steps"] > 10
    assert evaluate(m, Xv, yv)["roc_auc"] > 0.9


def test_train_logistic_gpu_graph(data):
    X, y, Xv, yv = data
    m, info = train_logistic(X, y, TrainConfig(epochs=3, lr=3e-2, batch=4096, device="cuda", graph=True))
    assert info.get("graph") is True
    assert evaluate(m, Xv, yv)["roc_auc"] > 0.9
