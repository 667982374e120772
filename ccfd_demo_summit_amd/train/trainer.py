"""Model training (replaces the JupyterHub/Spark workbench of the reference,
deploy/frauddetection_cr.yaml:7-53).

* ``train_logistic`` / ``train_mlp``: PyTorch-ROCm training on the GPU (bf16 autocast for
  the MLP, class-imbalance weighting), optionally data-parallel with DDP over RCCL when
  launched under torchrun.  The result is exported into the same ``LogisticModel`` /
  ``MLPModel`` containers the HIP kernels consume, so a trained model is packed and
  hot-swapped exactly like a random-init one.
* ``train_oblivious_gbdt``: gradient-boosted oblivious trees (logloss, second-order
  leaves, quantile-binned splits) with histograms built by ``scatter_add`` on the GPU.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Dict, Optional, Tuple

import numpy as np
import torch
import torch.nn as nn

from ..models.common import Normalizer
from ..models.gbdt import ObliviousGBDT
from ..models.lr import LogisticModel
from ..models.mlp import H1, H2, MLPModel


@dataclass
class TrainConfig:
    epochs: int = 3
    batch: int = 8192
    lr: float = 3e-3
    weight_decay: float = 1e-4
    pos_weight: Optional[float] = None     # default: sqrt(neg/pos)
    seed: int = 0
    device: str = "auto"
    bf16: bool = True
    metrics: Optional[object] = None       # metrics.exporter.TrainMetrics (Training dashboard)


def _device(name: str) -> torch.device:
    if name == "auto":
        return torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu")
    return torch.device(name)


def _ddp_ctx():
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def _fit(net: nn.Module, Xn: np.ndarray, y: np.ndarray, cfg: TrainConfig, use_bf16: bool) -> Dict[str, float]:
    dev = _device(cfg.device)
    torch.manual_seed(cfg.seed)
    rank, world = _ddp_ctx()
    net = net.to(dev)
    model = net
    if world > 1:
        from torch.nn.parallel import DistributedDataParallel as DDP
        model = DDP(net, device_ids=[dev.index] if dev.type == "cuda" else None)
    Xt = torch.from_numpy(np.ascontiguousarray(Xn)).to(dev)
    yt = torch.from_numpy(y.astype(np.float32)).to(dev)
    pos = float(y.sum())
    pw = cfg.pos_weight if cfg.pos_weight is not None else math.sqrt(max(1.0, (len(y) - pos) / max(pos, 1.0)))
    loss_fn = nn.BCEWithLogitsLoss(pos_weight=torch.tensor(pw, device=dev))
    opt = torch.optim.AdamW(model.parameters(), lr=cfg.lr, weight_decay=cfg.weight_decay)
    g = torch.Generator(device="cpu").manual_seed(cfg.seed)
    n = Xt.shape[0]
    shard = torch.arange(rank, n, world)
    steps = 0
    last = float("nan")
    tm = cfg.metrics
    name = "mlp" if isinstance(net, nn.Sequential) else "lr"
    if tm is not None:
        tm.workers.set(world)
    import time as _time
    t_start = _time.perf_counter()
    for _ in range(cfg.epochs):
        perm = shard[torch.randperm(len(shard), generator=g)].to(dev)
        for s in range(0, len(perm), cfg.batch):
            idx = perm[s:s + cfg.batch]
            with torch.autocast(device_type=dev.type, dtype=torch.bfloat16, enabled=use_bf16 and dev.type == "cuda"):
                logit = model(Xt[idx]).squeeze(-1)
            loss = loss_fn(logit.float(), yt[idx])
            opt.zero_grad(set_to_none=True)
            loss.backward()
            opt.step()
            steps += 1
            last = float(loss.detach())
            if tm is not None:
                tm.loss.labels(name).set(last)
                tm.steps.labels(name).inc()
                tm.samples_per_s.labels(name).set(steps * cfg.batch / max(1e-9, _time.perf_counter() - t_start))
                if dev.type == "cuda":
                    tm.mem_bytes.set(torch.cuda.memory_allocated(dev))
    return {"steps": steps, "final_loss": last, "pos_weight": pw}


def train_logistic(X: np.ndarray, y: np.ndarray, cfg: TrainConfig = TrainConfig()) -> Tuple[LogisticModel, Dict]:
    norm = Normalizer.fit(X)
    net = nn.Linear(X.shape[1], 1)
    with torch.no_grad():                 # convex problem: deterministic zero start
        net.weight.zero_()
        net.bias.zero_()
    info = _fit(net, norm(X), y, cfg, use_bf16=False)
    w = net.weight.detach().float().cpu().numpy()[0]
    b = float(net.bias.detach().float().cpu().numpy()[0])
    return LogisticModel(w.astype(np.float32), b, norm), info


def train_mlp(X: np.ndarray, y: np.ndarray, cfg: TrainConfig = TrainConfig()) -> Tuple[MLPModel, Dict]:
    norm = Normalizer.fit(X)
    torch.manual_seed(cfg.seed)           # reproducible init
    net = nn.Sequential(nn.Linear(X.shape[1], H1), nn.ReLU(), nn.Linear(H1, H2), nn.ReLU(), nn.Linear(H2, 1))
    info = _fit(net, norm(X), y, cfg, use_bf16=cfg.bf16)
    p = [t.detach().float().cpu().numpy() for t in net.parameters()]
    m = MLPModel(p[0], p[1], p[2], p[3], p[4][0], float(p[5][0]), norm)
    return m, info


# ---------------------------------------------------------------------------- GBDT
def _quantile_borders(X: np.ndarray, n_bins: int) -> np.ndarray:
    qs = np.linspace(0, 1, n_bins + 1)[1:-1]
    return np.quantile(X, qs, axis=0).T.astype(np.float32)        # [F, n_bins-1]


def train_oblivious_gbdt(X: np.ndarray, y: np.ndarray, n_trees: int = 100, depth: int = 6,
                         learning_rate: float = 0.1, n_bins: int = 32, l2: float = 1.0,
                         device: str = "auto") -> Tuple[ObliviousGBDT, Dict]:
    """Level-wise oblivious boosting on logloss.  At each level one (feature, border) is
    chosen for ALL current leaves (maximum summed second-order gain)."""
    dev = _device(device)
    X = np.asarray(X, np.float32)
    n, F = X.shape
    borders = _quantile_borders(X, n_bins)                          # [F, B-1]
    # bin index of every value: number of borders strictly below it -> x > border[b] iff bin > b
    bins = np.empty((n, F), np.int64)
    for f in range(F):
        bins[:, f] = np.searchsorted(borders[f], X[:, f], side="left")
    bt = torch.from_numpy(bins).to(dev)
    yt = torch.from_numpy(y.astype(np.float32)).to(dev)
    p0 = float(np.clip(y.mean(), 1e-6, 1 - 1e-6))
    base = math.log(p0 / (1 - p0))
    raw = torch.full((n,), base, device=dev)
    feat = np.zeros((n_trees, depth), np.int32)
    thr = np.zeros((n_trees, depth), np.float32)
    leaves = np.zeros((n_trees, 1 << depth), np.float32)
    B = n_bins
    fidx = torch.arange(F, device=dev)
    for t in range(n_trees):
        prob = torch.sigmoid(raw)
        grad = prob - yt
        hess = (prob * (1 - prob)).clamp_min(1e-6)
        leaf = torch.zeros(n, dtype=torch.long, device=dev)
        for d in range(depth):
            L = 1 << d
            key = (leaf[:, None] * F + fidx[None, :]) * B + bt          # [n, F]
            G = torch.zeros(L * F * B, device=dev).scatter_add_(0, key.reshape(-1), grad[:, None].expand(n, F).reshape(-1))
            H = torch.zeros(L * F * B, device=dev).scatter_add_(0, key.reshape(-1), hess[:, None].expand(n, F).reshape(-1))
            G = G.view(L, F, B)
            H = H.view(L, F, B)
            Gl = G.cumsum(-1)[..., :-1]                                # split after bin b: left = bins <= b
            Hl = H.cumsum(-1)[..., :-1]
            Gt = G.sum(-1, keepdim=True)
            Ht = H.sum(-1, keepdim=True)
            Gr, Hr = Gt - Gl, Ht - Hl
            gain = (Gl ** 2 / (Hl + l2) + Gr ** 2 / (Hr + l2) - Gt ** 2 / (Ht + l2)).sum(0)   # [F, B-1]
            best = int(torch.argmax(gain))
            f, b = divmod(best, B - 1)
            feat[t, d] = f
            thr[t, d] = borders[f, b]
            leaf = leaf | ((bt[:, f] > b).long() << d)
        Gs = torch.zeros(1 << depth, device=dev).scatter_add_(0, leaf, grad)
        Hs = torch.zeros(1 << depth, device=dev).scatter_add_(0, leaf, hess)
        vals = -learning_rate * Gs / (Hs + l2)
        leaves[t] = vals.cpu().numpy()
        raw = raw + vals[leaf]
    model = ObliviousGBDT(feat, thr, leaves, float(base))
    with torch.no_grad():
        ll = float(torch.nn.functional.binary_cross_entropy_with_logits(raw, yt))
    return model, {"train_logloss": ll, "trees": n_trees, "depth": depth}


def evaluate(model, X: np.ndarray, y: np.ndarray) -> Dict[str, float]:
    from sklearn.metrics import average_precision_score, roc_auc_score
    p = model.predict_proba(X)
    return {"roc_auc": float(roc_auc_score(y, p)), "pr_auc": float(average_precision_score(y, p))}
