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
    graph: bool = True                     # single GPU: replay the whole step as one HIP graph
    log_every: int = 50                    # graph mode: loss read back every N steps


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
    if cfg.graph and dev.type == "cuda" and world == 1 and len(shard) >= cfg.batch:
        return _fit_graph(model, Xt, yt, loss_fn, opt, shard, g, cfg, use_bf16, pw, name, tm, t_start)
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


def _fit_graph(model, Xt, yt, loss_fn, opt, shard, g, cfg: TrainConfig, use_bf16: bool, pw: float, name: str,
               tm, t_start) -> Dict[str, float]:
    """The training step (gather -> forward -> BCE -> backward -> AdamW) captured once as a
    HIP graph (``torch.cuda.CUDAGraph`` is hipGraph on ROCm) and replayed per step.  A
    12K-parameter MLP step is ~40 tiny kernels, i.e. launch-bound; a replay is one launch,
    plus one index copy into the static batch-index buffer.  Batches are full ``cfg.batch``
    rows (the tail of an epoch that does not fill one is skipped), the optimizer state lives
    in capturable tensors, and the loss is read back only every ``cfg.log_every`` steps."""
    import time as _time
    dev = Xt.device
    B = cfg.batch
    for group in opt.param_groups:         # optimizer step must run inside the graph
        group["capturable"] = True
    idx = torch.zeros(B, dtype=torch.int64, device=dev)
    xb = torch.empty(B, Xt.shape[1], dtype=Xt.dtype, device=dev)
    yb = torch.empty(B, dtype=yt.dtype, device=dev)

    def step():
        torch.index_select(Xt, 0, idx, out=xb)
        torch.index_select(yt, 0, idx, out=yb)
        with torch.autocast(device_type="cuda", dtype=torch.bfloat16, enabled=use_bf16, cache_enabled=False):
            logit = model(xb).squeeze(-1)
        loss = loss_fn(logit.float(), yb)
        loss.backward()
        opt.step()
        return loss

    batches = []
    for _ in range(cfg.epochs):
        perm = shard[torch.randperm(len(shard), generator=g)].to(dev)
        batches += [perm[s:s + B] for s in range(0, len(perm) - B + 1, B)]
    # warm-up (real steps on the first batches) on a side stream, as capture requires
    warm = min(3, len(batches))
    side = torch.cuda.Stream(dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(side):
        for k in range(warm):
            idx.copy_(batches[k])
            opt.zero_grad(set_to_none=False)
            step()
    torch.cuda.current_stream(dev).wait_stream(side)
    graph = torch.cuda.CUDAGraph()
    opt.zero_grad(set_to_none=False)        # grads stay allocated: the graph accumulates into them
    with torch.cuda.graph(graph):
        for p in model.parameters():
            p.grad.zero_()
        static_loss = step()
    last = float("nan")
    steps = logged = warm
    for k in range(warm, len(batches)):
        idx.copy_(batches[k], non_blocking=True)
        graph.replay()
        steps += 1
        if tm is not None and (steps % cfg.log_every == 0 or k == len(batches) - 1):
            last = float(static_loss.detach())
            tm.loss.labels(name).set(last)
            tm.steps.labels(name).inc(steps - logged)
            logged = steps
            tm.samples_per_s.labels(name).set(steps * B / max(1e-9, _time.perf_counter() - t_start))
            tm.mem_bytes.set(torch.cuda.memory_allocated(dev))
    torch.cuda.synchronize(dev)
    last = float(static_loss.detach()) if len(batches) > warm else last
    return {"steps": steps, "final_loss": last, "pos_weight": pw, "graph": True,
            "seconds": _time.perf_counter() - t_start}


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
                         device: str = "auto", borders: Optional[np.ndarray] = None) -> Tuple[ObliviousGBDT, Dict]:
    """Level-wise oblivious boosting on logloss.  At each level one (feature, border) is
    chosen for ALL current leaves (maximum summed second-order gain).

    Data-parallel when torch.distributed is initialised (the reference's 2-executor Spark
    training, deploy/frauddetection_cr.yaml:27,34-35): like the DDP trainers every rank
    passes the same X and works on its shard (rows rank::world); the borders come from
    rank 0 (broadcast), and the per-level gradient/hessian histograms,
    the leaf sums and the base-rate statistics are all-reduced (SUM), so every rank grows
    the same trees -- the ones a single process would grow on the union of the shards, up to
    float summation order.  ``borders`` [F, n_bins-1]: use these split candidates instead of
    quantiles of X."""
    dev = _device(device)
    rank, world = _ddp_ctx()

    def allreduce(t: torch.Tensor) -> torch.Tensor:
        if world > 1:
            import torch.distributed as dist
            dist.all_reduce(t)
        return t

    X = np.asarray(X, np.float32)
    if borders is None:
        borders = _quantile_borders(X, n_bins)                      # [F, B-1]
    if world > 1:
        X, y = X[rank::world], np.asarray(y)[rank::world]
    n, F = X.shape
    borders = np.ascontiguousarray(borders, np.float32)
    n_bins = borders.shape[1] + 1
    if world > 1:                                                   # rank 0's split candidates
        import torch.distributed as dist
        bt0 = torch.from_numpy(borders).to(dev)
        dist.broadcast(bt0, 0)
        borders = bt0.cpu().numpy()
    # bin index of every value: number of borders strictly below it -> x > border[b] iff bin > b
    bins = np.empty((n, F), np.int64)
    for f in range(F):
        bins[:, f] = np.searchsorted(borders[f], X[:, f], side="left")
    bt = torch.from_numpy(bins).to(dev)
    yt = torch.from_numpy(y.astype(np.float32)).to(dev)
    stats = allreduce(torch.tensor([float(y.sum()), float(n)], dtype=torch.float64, device=dev))
    p0 = float(np.clip(float(stats[0]) / max(float(stats[1]), 1.0), 1e-6, 1 - 1e-6))
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
            G = allreduce(G).view(L, F, B)
            H = allreduce(H).view(L, F, B)
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
        Gs = allreduce(torch.zeros(1 << depth, device=dev).scatter_add_(0, leaf, grad))
        Hs = allreduce(torch.zeros(1 << depth, device=dev).scatter_add_(0, leaf, hess))
        vals = -learning_rate * Gs / (Hs + l2)
        leaves[t] = vals.cpu().numpy()
        raw = raw + vals[leaf]
    model = ObliviousGBDT(feat, thr, leaves, float(base))
    with torch.no_grad():
        ll_sum = torch.nn.functional.binary_cross_entropy_with_logits(raw, yt, reduction="sum").double()
        ll = float(allreduce(ll_sum.reshape(1))[0]) / max(float(stats[1]), 1.0)
    return model, {"train_logloss": ll, "trees": n_trees, "depth": depth, "world": world}


def evaluate(model, X: np.ndarray, y: np.ndarray) -> Dict[str, float]:
    from sklearn.metrics import average_precision_score, roc_auc_score
    p = model.predict_proba(X)
    return {"roc_auc": float(roc_auc_score(y, p)), "pr_auc": float(average_precision_score(y, p))}
