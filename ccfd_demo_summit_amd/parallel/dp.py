"""Data-parallel stream sharding over RCCL.

One process per GPU (rank r of W).  The reference's only scale-out knobs are pod
``replicas`` and Kafka partitions (deploy/model/modelfull.json:46,
deploy/frauddetection_cr.yaml:76); here:

* partitions ``p`` with ``p % W == r`` belong to rank r (consumer-group assignment);
* X1: the packed model blob is **broadcast** from rank 0 at load and at hot swap, and
  verified bit-identical with a checksum all-reduce;
* X2: each rank's device counters (cumulative u64 slots, csrc/include/ccfd_abi.h) are
  **all-reduced** on a low-priority side stream once per epoch, overlapped with scoring
  (the engine flips to the other epoch buffer first, so the reduction never races the
  scoring kernels' atomics);
* X3: per-rank log2 latency histograms are merged by the same all-reduce (a histogram
  sum IS the merged sketch) -- one small collective per period instead of three.

Backend ``nccl`` on ROCm is RCCL over xGMI; CPU tests use ``gloo`` with the same code.
All messages are < 1 KB, so these collectives are latency-bound: one per period.
"""
from __future__ import annotations

import datetime
import os
import warnings
from dataclasses import dataclass
from typing import List, Optional

import numpy as np
import torch
import torch.distributed as dist

N_COUNTER_SLOTS = 64
N_LAT_BUCKETS = 256


@dataclass
class DistContext:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    device: torch.device = torch.device("cpu")
    backend: str = "none"

    @property
    def initialized(self) -> bool:
        return (self.world > 1 or self.backend != "none") and dist.is_initialized()


def init_distributed(backend: Optional[str] = None, timeout_s: float = 600.0) -> DistContext:
    """Initialise from torchrun env (RANK/WORLD_SIZE/LOCAL_RANK/MASTER_ADDR/PORT)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # Rehearsal knobs (never needed in production): CCFD_DIST_BACKEND=gloo runs the
    # collectives over gloo while the engines stay on the GPU, and CCFD_DEVICE_MODULO=1 maps
    # local rank r to GPU r % device_count, so a multi-rank job can be exercised on a box
    # with fewer GPUs than ranks (RCCL itself refuses two ranks on one GPU).
    # CCFD_FORCE_PG=1 builds the process group even at WORLD_SIZE=1, so a one-GPU box runs
    # the real RCCL collectives (X1/X2/X3 kernels next to the persistent scoring kernel).
    backend = backend or os.environ.get("CCFD_DIST_BACKEND") or None
    gpu_ok = torch.cuda.is_available()
    use_gpu = gpu_ok and (backend != "gloo" or os.environ.get("CCFD_DIST_BACKEND") == "gloo")
    if use_gpu:
        n_dev = torch.cuda.device_count()
        if os.environ.get("CCFD_DEVICE_MODULO") == "1":
            local = local % max(1, n_dev)
        elif local >= n_dev:
            raise RuntimeError(f"LOCAL_RANK {local} but this node has {n_dev} visible GPU(s): one rank per "
                               "GPU (a rehearsal shares them: bench.py --rehearsal / CCFD_DEVICE_MODULO=1)")
        torch.cuda.set_device(local)
        device = torch.device("cuda", local)
    else:
        device = torch.device("cpu")
    force = os.environ.get("CCFD_FORCE_PG") == "1"
    if (world > 1 or force) and not dist.is_initialized():
        be = backend or ("nccl" if use_gpu else "gloo")
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        kw = dict(backend=be, rank=rank, world_size=world, timeout=datetime.timedelta(seconds=timeout_s))
        if be == "nccl":
            kw["device_id"] = device
        dist.init_process_group(**kw)
        return DistContext(rank, world, local, device, be)
    return DistContext(rank, world, local, device, "none")


def x_group(ctx: DistContext):
    """A second process group over all ranks for the collectives issued from an engine's
    scoring thread (X2 epochs, runtime X1).  torch.distributed pairs collectives by call
    order per group; giving the scoring thread its own group keeps its sequence independent
    of collectives the main thread issues (barriers, bench reductions).  Collective call:
    every rank creates it at the same point.  None when not distributed."""
    if not ctx.initialized:
        return None
    return dist.new_group(ranks=list(range(ctx.world)))


def assign_partitions(n_partitions: int, rank: int, world: int) -> List[int]:
    """Static consumer-group assignment: partition p -> rank p % world."""
    return [p for p in range(n_partitions) if p % world == rank]


def broadcast_blob(ctx: DistContext, blob: Optional[torch.Tensor], src: int = 0, group=None) -> torch.Tensor:
    """X1: rank ``src`` sends its packed model blob (uint8, on ctx.device) to every rank and
    every rank verifies the received bytes against the sender's checksum.  ``group``: the
    process group (the engine thread's X-group at runtime, see ``x_group``)."""
    if not ctx.initialized:
        assert blob is not None
        return blob
    n = torch.tensor([blob.numel() if ctx.rank == src else 0], dtype=torch.int64, device=ctx.device)
    dist.broadcast(n, src, group=group)
    if ctx.rank != src:
        blob = torch.empty(int(n.item()), dtype=torch.uint8, device=ctx.device)
    dist.broadcast(blob, src, group=group)
    ck = _checksum(blob)
    lo, hi = ck.clone(), ck.clone()
    dist.all_reduce(lo, op=dist.ReduceOp.MIN, group=group)
    dist.all_reduce(hi, op=dist.ReduceOp.MAX, group=group)
    if not torch.equal(lo, hi):
        raise RuntimeError("model blob broadcast mismatch between ranks")
    return blob


def resolve_row_format(kind: str, wire: str = "auto") -> str:
    """Partition-log row format of a model kind: ``auto`` = W64 for the MLP / LR kernels,
    G20 for GBDT (the PCIe-byte-optimal exact or bf16 formats, contracts/transaction.py;
    ``broadcast_model`` widens G20 -> G32 -> f32 when an ensemble's bin table needs it)."""
    if wire == "auto":
        return "g20" if kind == "gbdt" else "w64"
    if (wire == "w64" and kind == "gbdt") or (wire in ("g32", "g20") and kind != "gbdt"):
        raise ValueError(f"row format {wire} does not apply to model kind {kind}")
    return wire


def broadcast_model(ctx: DistContext, model, kind: str, row_format: str, group=None):
    """X1 for a whole device model: rank 0 packs ``model`` for ``row_format`` (f32 / w64 /
    g32) and broadcasts the blob -- plus, for G32, the bin table every rank encodes its
    partition logs with, and the tree shape; every rank returns an equal DeviceModel.
    ``model`` is only read on rank 0.

    G20 needs at most 31 distinct split thresholds per feature (5-bit bins), G32 at most 255
    (u8 bins).  An ensemble with more widens to the next format (G20 -> G32 -> f32 rows) on
    every rank: rank 0 decides and the decision travels in the header broadcast ahead of
    the blob, so all ranks agree.  Callers take the row format from the returned model
    (``DeviceModel.row_format``)."""
    from ..models.gbdt import BinSpec
    from ..ops.kernels import DeviceModel
    codes = {"f32": 0, "w64": 1, "g32": 2, "g20": 3}
    blob = spec_t = None
    header = torch.zeros(3, dtype=torch.int64, device=ctx.device)      # trees, depth, row format
    if ctx.rank == 0:
        fmt = row_format
        if fmt == "g20":
            try:
                spec = model.bin_spec(bits=5)
            except ValueError as e:                 # > 31 thresholds on a feature
                warnings.warn(f"G20 rows impossible for this ensemble ({e}); trying G32 rows")
                fmt = "g32"
        if fmt == "g32":
            try:
                spec = model.bin_spec()
            except ValueError as e:                 # > 255 thresholds on a feature
                warnings.warn(f"G32 rows impossible for this ensemble ({e}); scoring f32 rows")
                fmt = "f32"
        if fmt in ("g32", "g20"):
            packed = model.pack(bins=spec)
            spec_t = torch.from_numpy(np.frombuffer(spec.to_bytes(), np.uint8).copy()).to(ctx.device)
        else:
            packed = model.pack(wire=True) if fmt == "w64" else model.pack()
        blob = torch.from_numpy(np.frombuffer(packed, np.uint8).copy()).to(ctx.device)
        header[0], header[1] = getattr(model, "n_trees", 0), getattr(model, "depth", 0)
        header[2] = codes[fmt]
    if ctx.initialized:
        dist.broadcast(header, 0, group=group)
    fmt = {v: k for k, v in codes.items()}[int(header[2])]
    blob = broadcast_blob(ctx, blob, group=group)
    bins = None
    if fmt in ("g32", "g20"):
        bins = BinSpec.from_bytes(broadcast_blob(ctx, spec_t, group=group).cpu().numpy().tobytes(),
                                  bits=8 if fmt == "g32" else 5)
    return DeviceModel.from_blob(kind, blob, int(header[0]), int(header[1]), wire=fmt == "w64", bins=bins)


def _checksum(blob: torch.Tensor) -> torch.Tensor:
    b = blob.to(torch.int64)
    idx = torch.arange(b.numel(), device=b.device, dtype=torch.int64)
    return torch.stack([b.sum(), (b * (idx % 65521 + 1)).sum()])


N_CTRL_SLOTS = 4      # control words carried by the same all-reduce (hot-swap header)
_K = N_COUNTER_SLOTS + N_LAT_BUCKETS


class CounterReducer:
    """X2/X3: periodic all-reduce of epoch counter buffers + latency histograms.

    ``submit(closed, lat_hist, ctrl)`` enqueues on the side stream: copy the counters, the
    latency histogram and ``N_CTRL_SLOTS`` control words into one packed vector, zero the
    closed epoch buffer (event ``freed``: a LOCAL dependency only), then start the all-reduce
    (sum) ASYNCHRONOUSLY.  ``complete()`` folds the result into ``totals``; ``busy()`` says
    whether the reduction is still waiting for other ranks.  Nothing here makes the host wait
    for a remote rank unless it asks to (``complete()`` on a busy reducer)."""

    def __init__(self, ctx: DistContext, device: torch.device, priority: int = 0, group=None):
        self.ctx = ctx
        self.device = device
        self.group = group
        self.totals = torch.zeros(_K, dtype=torch.int64, device=device)
        self.local_totals = torch.zeros_like(self.totals)
        self.pack = torch.zeros(_K + N_CTRL_SLOTS, dtype=torch.int64, device=device)
        self.side = torch.cuda.Stream(device, priority=priority) if device.type == "cuda" else None
        self.done = torch.cuda.Event() if device.type == "cuda" else None
        self.freed = torch.cuda.Event() if device.type == "cuda" else None
        self.epochs = 0
        self._work = None
        self.last_ctrl: Optional[torch.Tensor] = None     # reduced control words of the last completion
        # At world 1 RCCL elides the in-place int64 SUM entirely (no device kernel, measured:
        # profiles/r3/x2_overlap/).  CCFD_X2_ONE_RANK_KERNEL=1 (evidence runs on a one-GPU box
        # only) adds, per X2 tick, one float32 AVG all-reduce of the same size on the same
        # communicator -- RCCL runs that as its oneRankReduce device kernel on the
        # communicator's stream -- so a kernel trace shows where an X2 reduction kernel
        # executes relative to the resident scoring kernel
        self._op = dist.ReduceOp.SUM
        self._kernel_probe = None
        self._probe_work = None
        if os.environ.get("CCFD_X2_ONE_RANK_KERNEL") == "1" and ctx.world == 1 and ctx.initialized:
            self._kernel_probe = torch.ones(_K + N_CTRL_SLOTS, dtype=torch.float32, device=device)

    def busy(self) -> bool:
        return self._work is not None and not self._work.is_completed()

    def submit(self, closed: torch.Tensor, lat_hist: Optional[np.ndarray] = None,
               ctrl: Optional[np.ndarray] = None) -> None:
        self.complete()                                  # at most one reduction in flight
        ctxm = torch.cuda.stream(self.side) if self.side is not None else _nullctx()
        with ctxm:
            self.pack[:N_COUNTER_SLOTS].copy_(closed, non_blocking=True)
            for lo, hi, v in ((N_COUNTER_SLOTS, _K, lat_hist), (_K, _K + N_CTRL_SLOTS, ctrl)):
                if v is None:
                    self.pack[lo:hi].zero_()
                    continue
                h = torch.from_numpy(np.ascontiguousarray(v, np.int64))
                if self.device.type == "cuda":
                    h = h.pin_memory()
                self.pack[lo:hi].copy_(h, non_blocking=True)
            self.local_totals += self.pack[:_K]
            closed.zero_()
            if self.freed is not None:
                self.freed.record(self.side)
            if self.ctx.initialized:
                self._work = dist.all_reduce(self.pack, op=self._op, group=self.group, async_op=True)
                if self._kernel_probe is not None:
                    self._probe_work = dist.all_reduce(self._kernel_probe, op=dist.ReduceOp.AVG,
                                                       group=self.group, async_op=True)
            else:
                self._fold()
        self.epochs += 1

    def _fold(self) -> None:
        self.totals += self.pack[:_K]
        self.last_ctrl = self.pack[_K:].clone()
        if self.done is not None:
            self.done.record(self.side)

    def complete(self) -> None:
        """Fold the in-flight reduction into ``totals`` (blocks only if it is still running)."""
        if self._work is None:
            return
        ctxm = torch.cuda.stream(self.side) if self.side is not None else _nullctx()
        with ctxm:
            self._work.wait()            # RCCL: the side stream waits; gloo: the host waits
            self._work = None
            if self._probe_work is not None:
                self._probe_work.wait()
                self._probe_work = None
            self._fold()

    def pop_ctrl(self) -> Optional[np.ndarray]:
        if self.last_ctrl is None:
            return None
        if self.side is not None:
            self.side.synchronize()
        v, self.last_ctrl = self.last_ctrl.cpu().numpy(), None
        return v

    def wait(self) -> None:
        self.complete()
        if self.side is not None:
            self.side.synchronize()

    def snapshot(self):
        """(global counters u64[64], global latency histogram u64[256]) as numpy, as of the
        last completed reduction (does not wait for one still in flight)."""
        if self.side is not None:
            self.side.synchronize()
        t = self.totals.cpu().numpy()
        return t[:N_COUNTER_SLOTS], t[N_COUNTER_SLOTS:]

    def local_snapshot(self):
        if self.side is not None:
            self.side.synchronize()
        t = self.local_totals.cpu().numpy()
        return t[:N_COUNTER_SLOTS], t[N_COUNTER_SLOTS:]


class EpochPipeline:
    """Drives X2 for one engine: flip the counter epoch, and hand the CLOSED buffer to the
    CounterReducer only once every micro-batch of that epoch has completed (in the
    persistent exec mode there is no per-batch event a stream could wait on, so the host
    observes completion records instead).  One epoch of slack: the epoch closed at tick i is
    reduced at tick i+1, so the completion wait is empty in steady state.

    Pairing rule (ranks tick on their own clocks): every tick that runs issues exactly one
    collective (none on the first), and a rank never issues its next one before its previous
    one completed -- so tick counts of any two ranks differ by at most one, and
    ``tick(block=False)`` returns False instead of waiting when the previous reduction is
    still waiting for a slower rank.  ``ctrl``: optional object with ``contribute() ->
    int64[N_CTRL_SLOTS]`` and ``on_reduced(int64[N_CTRL_SLOTS])`` riding in the same
    all-reduce (the hot-swap header, parallel/hotswap.py)."""

    def __init__(self, engine, reducer: CounterReducer, ctrl=None):
        self.engine = engine
        self.reducer = reducer
        self.ctrl = ctrl
        self.pending = None          # (buffer, flip_count, lat_delta)
        self.ticks = 0

    def _progress_until(self, cond, progress, timeout_s: float, what: str) -> None:
        import time as _t
        t0 = _t.monotonic()
        while not cond():
            if progress is not None:
                progress()
            if _t.monotonic() - t0 > timeout_s:
                raise TimeoutError(what)

    def _complete(self) -> None:
        self.reducer.complete()
        if self.ctrl is None:
            self.reducer.last_ctrl = None
            return
        v = self.reducer.pop_ctrl()
        if v is not None:
            self.ctrl.on_reduced(v)

    def tick(self, lat_delta=None, progress=None, timeout_s: float = 60.0, block: bool = True) -> bool:
        """One X2 step; returns False (nothing done) when ``block`` is False and the previous
        reduction has not completed yet."""
        if self.reducer.busy():
            if not block:
                return False
            self._progress_until(lambda: not self.reducer.busy(), progress, timeout_s,
                                 "X2 all-reduce did not complete: a peer rank stopped ticking")
        if not block and self.pending is not None and not self.engine.epoch_complete(self.pending[1]):
            # the closed epoch still has batches in flight -- or the engine is HELD (hand-off
            # back-pressure: the serving thread retires nothing until the caller's next step
            # releases it), so waiting here would wait for the caller itself: skip the tick
            return False
        self._complete()
        self.ticks += 1
        if self.pending is not None:
            self._progress_until(lambda: self.engine.epoch_complete(self.pending[1]), progress, timeout_s,
                                 "epoch did not complete: engine stalled")
            ctrl = self.ctrl.contribute() if self.ctrl is not None else None
            self.reducer.submit(self.pending[0], self.pending[2], ctrl)
            self.pending = None
            if self.reducer.freed is not None:
                self.reducer.freed.synchronize()    # local: the buffer reopened below is zeroed
        buf = self.engine.flip_epoch(self.reducer.side)
        self.pending = (buf, self.engine.flips, lat_delta)
        return True

    def finish(self, progress=None, timeout_s: float = 60.0) -> None:
        """Call after the engine has drained (collective, same program point on every rank):
        reduce the last closed AND the open epoch."""
        self._complete()
        if self.pending is not None:
            self._progress_until(lambda: self.engine.epoch_complete(self.pending[1]), progress, timeout_s,
                                 "epoch did not complete: engine stalled")
            self.reducer.submit(self.pending[0], self.pending[2])
            self.pending = None
        self._complete()
        if self.reducer.freed is not None:
            self.reducer.freed.synchronize()
        self.reducer.submit(self.engine.flip_epoch(self.reducer.side), None)
        self._complete()
        self.reducer.wait()


class _nullctx:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def hist_quantile(hist: np.ndarray, q: float, per_octave: int = 4) -> float:
    """Quantile (in the histogram's unit, ns) of a log-bucket histogram: bucket i holds
    values in [2^(i/k), 2^((i+1)/k)), k = per_octave; geometric interpolation inside."""
    hist = np.asarray(hist, np.float64)
    tot = hist.sum()
    if tot <= 0:
        return 0.0
    target = q * tot
    c = np.cumsum(hist)
    i = int(np.searchsorted(c, target, side="left"))
    i = min(i, len(hist) - 1)
    prev = c[i - 1] if i > 0 else 0.0
    frac = (target - prev) / max(hist[i], 1.0)
    return float(2.0 ** ((i + frac) / per_octave))


def all_max(ctx: DistContext, value: float) -> float:
    if not ctx.initialized:
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=ctx.device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def all_sum(ctx: DistContext, value: float) -> float:
    if not ctx.initialized:
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=ctx.device)
    dist.all_reduce(t)
    return float(t.item())


def barrier(ctx: DistContext) -> None:
    if ctx.initialized:
        if ctx.backend == "nccl":
            dist.barrier(device_ids=[ctx.device.index])
        else:
            dist.barrier()
