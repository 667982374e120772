"""Python API over the fused HIP scoring kernels (csrc/kernels/*.hip).

All functions take torch tensors on the GPU and enqueue on the current torch stream.
There is deliberately NO silent fallback: on a machine with a GPU these ops either run
the gfx950 code object or raise (the CPU oracles live in ``models/*.py``).
"""
from __future__ import annotations

import ctypes as C
from typing import Optional, Tuple

import numpy as np
import torch

from ._lib import MODEL_IDS, N_COUNTER_SLOTS, ScoreArgs, check, lib

N_FEATURES = 30


class DeviceModel:
    """A packed model resident in HBM (the blob is broadcast once over RCCL in DP runs)."""

    def __init__(self, model, device: torch.device | str | int = "cuda", wire: bool = False):
        """``wire=True``: blob packed for W64 wire rows (MLP / LR; see contracts/transaction.py)."""
        self.kind = model.kind
        if self.kind not in MODEL_IDS:
            raise ValueError(f"no device kernel for model kind {self.kind!r}")
        if wire and self.kind not in ("mlp", "lr"):
            raise ValueError("W64 wire rows are supported by the MLP and LR kernels")
        self.wire = bool(wire)
        blob = np.frombuffer(model.pack(wire=True) if wire else model.pack(), np.uint8)
        self.blob = torch.from_numpy(blob.copy()).to(device)
        self.trees = getattr(model, "n_trees", 0)
        self.depth = getattr(model, "depth", 0)

    @classmethod
    def from_blob(cls, kind: str, blob: torch.Tensor, trees: int = 0, depth: int = 0,
                  wire: bool = False) -> "DeviceModel":
        self = cls.__new__(cls)
        self.kind, self.blob, self.trees, self.depth, self.wire = kind, blob, trees, depth, bool(wire)
        return self

    @property
    def model_id(self) -> int:
        return MODEL_IDS[self.kind]


class DeviceRules:
    """A compiled routing rule set resident in HBM (``RuleSet.device_program``); pass it to
    ``score(..., rules=)`` / ``StreamEngine(rules=)`` and the kernels' epilogue routes by the
    rules instead of ``proba >= threshold``."""

    def __init__(self, ruleset, device: torch.device | str | int = "cuda"):
        self.ruleset = ruleset
        prog = np.frombuffer(ruleset.device_program(), np.uint8)
        self.prog = torch.from_numpy(prog.copy()).to(device)

    @property
    def ptr(self) -> int:
        return self.prog.data_ptr()


def new_counters(device="cuda") -> torch.Tensor:
    return torch.zeros(N_COUNTER_SLOTS, dtype=torch.int64, device=device)


def score(dm: DeviceModel, x: torch.Tensor, threshold: float = 0.5,
          proba: Optional[torch.Tensor] = None, route: Optional[torch.Tensor] = None,
          counters: Optional[torch.Tensor] = None, stream: Optional[torch.cuda.Stream] = None,
          flags: int = 0, rules: Optional[DeviceRules] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """Fused score of x [n,30] (float32, CUDA) -- or, for a ``wire`` model, W64 rows
    ([n,64] uint8 or [n,16] float32 view) -- returns (proba_1 [n] f32, route [n] u8).
    ``flags``: extra ``CCFD_ARG_*`` bits (ablation switches for profiling)."""
    wire = getattr(dm, "wire", False)
    if wire:
        if not x.is_cuda or x.dim() != 2 or x.element_size() * x.shape[1] != 64 or not x.is_contiguous():
            raise ValueError("wire model: x must be contiguous CUDA W64 rows ([n,64] u8 / [n,16] f32)")
    elif not x.is_cuda or x.dtype != torch.float32 or x.dim() != 2 or x.shape[1] != N_FEATURES:
        raise ValueError("x must be a CUDA float32 tensor of shape [n, 30]")
    if x.stride(1) != 1:
        x = x.contiguous()
    n = x.shape[0]
    if proba is None:
        proba = torch.empty(n, dtype=torch.float32, device=x.device)
    if route is None:
        route = torch.empty(n, dtype=torch.uint8, device=x.device)
    a = ScoreArgs()
    a.x = x.data_ptr()
    a.ld = 16 if wire else x.stride(0)
    a.flags = (2 if wire else 0) | int(flags)          # CCFD_ARG_WIRE_W64
    a.n = n
    a.model = dm.model_id
    a.blob = dm.blob.data_ptr()
    a.threshold = float(threshold)
    a.gbdt_trees = dm.trees
    a.gbdt_depth = dm.depth
    a.proba = proba.data_ptr()
    a.route = route.data_ptr()
    a.counters = counters.data_ptr() if counters is not None else None
    a.rules = rules.ptr if rules is not None else None
    s = stream if stream is not None else torch.cuda.current_stream(x.device)
    check(lib().ccfd_score_launch(C.byref(a), C.c_void_p(s.cuda_stream)), "ccfd_score_launch")
    return proba, route
