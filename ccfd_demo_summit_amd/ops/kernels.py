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

from ._lib import (ARG_WIRE_G20, ARG_WIRE_G32, ARG_WIRE_W64, BIN_FORMATS, MODEL_IDS, N_COUNTER_SLOTS, ScoreArgs,
                   check, lib)

N_FEATURES = 30
ROW_BYTES = {"f32": 4 * N_FEATURES, "w64": 64, "g32": 32, "g20": 20}
WIRE_FLAGS = {"f32": 0, "w64": ARG_WIRE_W64, "g32": ARG_WIRE_G32, "g20": ARG_WIRE_G32 | ARG_WIRE_G20}


class DeviceModel:
    """A packed model resident in HBM (the blob is broadcast once over RCCL in DP runs)."""

    def __init__(self, model, device: torch.device | str | int = "cuda", wire: bool = False, bins=None):
        """``wire=True``: blob packed for W64 wire rows (MLP / LR; see contracts/transaction.py).
        ``bins``: GBDT on binned rows -- ``True`` for the model's own G32 bin table, ``"g20"``
        for the same table on 20-byte G20 rows (<= 31 thresholds a feature), or a
        ``models.gbdt.BinSpec`` containing its thresholds (e.g. the live logs' spec; its
        ``bits`` select G32 or G20)."""
        self.kind = model.kind
        if self.kind not in MODEL_IDS:
            raise ValueError(f"no device kernel for model kind {self.kind!r}")
        if wire and self.kind not in ("mlp", "lr"):
            raise ValueError("W64 wire rows are supported by the MLP and LR kernels")
        if bins is not None and bins is not False and self.kind != "gbdt":
            raise ValueError("G32 rows (bins=) are for the GBDT kernel")
        self.wire = bool(wire)
        if bins is True or bins == "g32":
            bins = model.bin_spec()
        elif isinstance(bins, str) and bins == "g20":
            bins = model.bin_spec(bits=5)
        self.bins = bins if bins is not False else None
        if self.bins is not None:
            packed = model.pack(bins=self.bins)
        else:
            packed = model.pack(wire=True) if wire else model.pack()
        self.blob = torch.from_numpy(np.frombuffer(packed, np.uint8).copy()).to(device)
        self.trees = getattr(model, "n_trees", 0)
        self.depth = getattr(model, "depth", 0)

    @classmethod
    def from_blob(cls, kind: str, blob: torch.Tensor, trees: int = 0, depth: int = 0,
                  wire: bool = False, bins=None) -> "DeviceModel":
        self = cls.__new__(cls)
        self.kind, self.blob, self.trees, self.depth, self.wire = kind, blob, trees, depth, bool(wire)
        self.bins = bins
        return self

    @property
    def model_id(self) -> int:
        return MODEL_IDS[self.kind]

    @property
    def row_format(self) -> str:
        """Row layout the blob expects: "f32" (30 x f32), "w64", "g32" or "g20"."""
        bins = getattr(self, "bins", None)
        return bins.row_format if bins is not None else "w64" if self.wire else "f32"


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
    ([n,64] uint8 or [n,16] float32 view), for a ``bins`` model G32 / G20 rows ([n,32] / [n,20] u8) --
    returns (proba_1 [n] f32, route [n] u8).
    ``flags``: extra ``CCFD_ARG_*`` bits (ablation switches for profiling)."""
    fmt = dm.row_format
    wire = fmt != "f32"
    if wire:
        rb = ROW_BYTES[fmt]
        if not x.is_cuda or x.dim() != 2 or x.element_size() * x.shape[1] != rb or not x.is_contiguous():
            raise ValueError(f"{fmt} model: x must be contiguous CUDA {fmt.upper()} rows ([n,{rb}] u8)")
        if fmt in BIN_FORMATS and rules is not None and rules.ruleset.feature_vars():
            raise ValueError("G32 / G20 rows carry bins, not feature values: routing rules may only use proba_1")
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
    a.ld = ROW_BYTES[fmt] // 4 if wire else x.stride(0)
    a.flags = WIRE_FLAGS[fmt] | int(flags)
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
