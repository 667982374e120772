"""Distributed path on CPU: gloo, world_size 2 (SURVEY.md §4.1 "Distributed without a
cluster"): broadcast weights bit-identical, all-reduced counters == global truth."""
import os
import socket
import time

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from ccfd_demo_summit_amd.parallel import assign_partitions, hist_quantile


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    from ccfd_demo_summit_amd.models import build_model
    from ccfd_demo_summit_amd.parallel import CounterReducer, broadcast_blob, init_distributed
    ctx = init_distributed(backend="gloo")
    try:
        blob = None
        if ctx.rank == 0:
            blob = torch.from_numpy(np.frombuffer(build_model("mlp", seed=9).pack(), np.uint8).copy())
        blob = broadcast_blob(ctx, blob)
        red = CounterReducer(ctx, torch.device("cpu"))
        # each rank scores a different number of rows per epoch
        for epoch in range(3):
            c = torch.zeros(64, dtype=torch.int64)
            c[0] = 1000 * (rank + 1) + epoch
            c[1] = rank + 1
            red.submit(c, np.full(256, rank + 1, np.int64))
            assert int(c.sum()) == 0          # epoch buffer zeroed for reuse
        red.wait()                            # fold the last (async) reduction
        g, lat = red.snapshot()
        q.put((rank, bytes(blob.numpy()), g[:2].tolist(), int(lat.sum())))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4, 8])
def test_gloo_broadcast_and_counter_allreduce(world):
    """W ranks on one node (W in {2,4,8}) through the same dist/ code path."""
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    from ccfd_demo_summit_amd.models import build_model
    want = build_model("mlp", seed=9).pack()
    assert all(r[1] == want for r in res)         # bit-identical weights on every rank
    truth0 = sum(1000 * (r + 1) + e for r in range(world) for e in range(3))
    ranks_sum = world * (world + 1) // 2
    for _, _, g, lat in res:
        assert g[0] == truth0 and g[1] == 3 * ranks_sum
        assert lat == 3 * 256 * ranks_sum


def test_assign_partitions_covers_each_once():
    for world in (1, 2, 3, 8):
        seen = []
        for r in range(world):
            seen += assign_partitions(16, r, world)
        assert sorted(seen) == list(range(16))


def test_hist_quantile():
    h = np.zeros(256, np.int64)
    # 100 samples in bucket of 2^10 ns (bucket index 40 at 4 per octave)
    h[40] = 100
    v = hist_quantile(h, 0.5)
    assert 2 ** 10 <= v < 2 ** 10.25
    assert hist_quantile(np.zeros(256), 0.5) == 0.0


class _FakeEngine:
    """Stands in for StreamEngine on CPU: records the blobs it is asked to swap to."""

    def __init__(self):
        from ccfd_demo_summit_amd.ops.kernels import DeviceModel
        self.wire = False
        self.dm = DeviceModel.from_blob("mlp", torch.zeros(16, dtype=torch.uint8))
        self.swapped = []

    def swap_model(self, dm):
        self.dm = dm
        self.swapped.append(bytes(dm.blob.numpy()))


def _hotswap_worker(rank, world, port, path, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    from ccfd_demo_summit_amd.models import build_model, save_model
    from ccfd_demo_summit_amd.parallel import init_distributed
    from ccfd_demo_summit_amd.parallel.hotswap import HotSwap
    ctx = init_distributed(backend="gloo")
    try:
        eng = _FakeEngine()
        hs = HotSwap(ctx, eng, watch_path=path if rank == 0 else None)
        got = [hs.tick()]                                   # nothing offered
        if rank == 0:
            hs.offer(build_model("mlp", seed=1))
        got.append(hs.tick())                               # explicit offer -> swap everywhere
        if rank == 0:
            import time
            time.sleep(0.05)
            save_model(build_model("mlp", seed=2), path)    # file watch -> second swap
            os.utime(path, (time.time() + 5, time.time() + 5))
        got.append(hs.tick())
        got.append(hs.tick())
        q.put((rank, got, hs.version, eng.swapped))
    finally:
        dist.destroy_process_group()


def test_hot_swap_broadcasts_new_weights(tmp_path):
    from ccfd_demo_summit_amd.models import build_model
    path = str(tmp_path / "model.safetensors")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_hotswap_worker, args=(r, 2, port, path, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(30)
    want = [build_model("mlp", seed=1).pack(), build_model("mlp", seed=2).pack()]
    for rank, got, version, swapped in res:
        assert got == [False, True, True, False], (rank, got)
        assert version == 2
        assert swapped == want


class _FakeEpochEngine(_FakeEngine):
    """CPU stand-in for the engine's epoch interface (two counter buffers, flip, completion)."""

    def __init__(self):
        super().__init__()
        self.counters = [torch.zeros(64, dtype=torch.int64), torch.zeros(64, dtype=torch.int64)]
        self.cur = 0
        self.flips = 0

    def flip_epoch(self, side=None):
        closed, self.cur = self.cur, self.cur ^ 1
        self.flips += 1
        return self.counters[closed]

    def epoch_complete(self, flip_count):
        return True

    def score(self, rows):
        self.counters[self.cur][0] += rows


def test_nonblocking_tick_skips_an_incomplete_epoch():
    """A held engine (hand-off back-pressure) retires nothing until the caller's next step
    releases it: a non-blocking tick must return instead of waiting for the closed epoch
    (the GPU back-pressure test stalled 60 s there), and tick once the epoch completed."""
    from ccfd_demo_summit_amd.parallel import CounterReducer, DistContext, EpochPipeline

    class Held(_FakeEpochEngine):
        done = False

        def epoch_complete(self, flip_count):
            return self.done
    eng = Held()
    ep = EpochPipeline(eng, CounterReducer(DistContext(0, 1, 0, torch.device("cpu"), "none"), torch.device("cpu")))
    assert ep.tick(block=False) and ep.ticks == 1          # opens the first epoch
    eng.score(10)
    t0 = time.monotonic()
    assert ep.tick(block=False) is False and ep.ticks == 1   # closed epoch incomplete: skipped
    assert time.monotonic() - t0 < 1.0
    eng.done = True
    assert ep.tick(block=False) and ep.ticks == 2
    ep.finish()


def _skewed_worker(rank, world, port, q):
    """Ranks tick on their own clocks (rank 0 five times, the others twice), then meet in a
    main-group barrier -- the shape that deadlocked when a tick blocked on its all-reduce --
    then flush: agree the tick count on a control group, catch up, finish."""
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    from ccfd_demo_summit_amd.models import build_model
    from ccfd_demo_summit_amd.parallel import CounterReducer, EpochPipeline, init_distributed, x_group
    from ccfd_demo_summit_amd.parallel.hotswap import HotSwap
    ctx = init_distributed(backend="gloo")
    try:
        xg, cg = x_group(ctx), x_group(ctx)
        eng = _FakeEpochEngine()
        hs = HotSwap(ctx, eng, group=xg)
        red = CounterReducer(ctx, torch.device("cpu"), group=xg)
        ep = EpochPipeline(eng, red, ctrl=hs)
        if rank == 0:
            hs.offer(build_model("mlp", seed=5))
        ran = []
        for _ in range(5 if rank == 0 else 2):
            eng.score(100 * (rank + 1))
            ran.append(ep.tick(block=False))
            hs.poll()
        dist.barrier()                                  # main thread meets the other ranks
        t = torch.tensor([ep.ticks], dtype=torch.int64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=cg)
        while ep.ticks < int(t):
            ep.tick(block=True)
        ep.finish()
        hs.poll(block=True)
        g, _ = red.snapshot()
        q.put((rank, ran, int(g[0]), hs.version, eng.swapped))
    finally:
        dist.destroy_process_group()


def test_skewed_ticks_never_block_and_flush_pairs():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_skewed_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(30)
        assert p.exitcode == 0
    from ccfd_demo_summit_amd.models import build_model
    truth = 5 * 100 + 2 * 200
    for rank, ran, total, version, swapped in res:
        assert total == truth, (rank, total)
        assert version == 1 and swapped == [build_model("mlp", seed=5).pack()]
    # rank 0 could not run ahead by more than one collective: later ticks were deferred
    assert res[0][1][:2] == [True, True] and False in res[0][1]


def _forced_worker(port, q):
    os.environ.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port), CCFD_FORCE_PG="1")
    import torch.distributed as dist
    from ccfd_demo_summit_amd.parallel import CounterReducer, all_max, init_distributed
    ctx = init_distributed(backend="gloo")
    try:
        red = CounterReducer(ctx, torch.device("cpu"))
        c = torch.zeros(64, dtype=torch.int64)
        c[0] = 7
        red.submit(c, np.ones(256, np.int64))
        red.wait()
        g, lat = red.snapshot()
        q.put((ctx.initialized, int(g[0]), int(lat.sum()), all_max(ctx, 1.5)))
    finally:
        dist.destroy_process_group()


def test_forced_process_group_at_world_one():
    """CCFD_FORCE_PG=1: a one-rank job still runs every collective (the one-GPU rehearsal of
    the N>1 bench path over real RCCL)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_forced_worker, args=(_free_port(), q))
    p.start()
    init, rows, lat, mx = q.get(timeout=120)
    p.join(timeout=60)
    assert p.exitcode == 0
    assert init and rows == 7 and lat == 256 and mx == 1.5


def _model_worker(rank, world, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    from ccfd_demo_summit_amd.data import generate
    from ccfd_demo_summit_amd.models import build_model
    from ccfd_demo_summit_amd.parallel import broadcast_model, init_distributed, resolve_row_format
    ctx = init_distributed(backend="gloo")
    try:
        out = {}
        X, _ = generate(4000, seed=5)
        for key, kind, wire in (("gbdt", "gbdt", "auto"), ("gbdt_g32", "gbdt", "g32"), ("mlp", "mlp", "auto")):
            fmt = resolve_row_format(kind, wire)
            m = build_model(kind, seed=3, X_ref=X) if ctx.rank == 0 else None
            dm = broadcast_model(ctx, m, kind, fmt)
            enc = dm.bins.encode(X[:100]).tobytes() if dm.bins is not None else b""
            out[key] = (fmt, bytes(dm.blob.numpy()), dm.trees, dm.depth, dm.row_format, enc)
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


def test_broadcast_model_carries_g32_bin_table():
    """X1 of a whole device model: every rank gets the same blob, tree shape and (G20 by
    default, or G32) bin table, so every rank encodes its own partition logs identically."""
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_model_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0] == res[1]
    fmt, blob, trees, depth, row_format, enc = res[0]["gbdt"]
    assert fmt == row_format == "g20" and blob[:4] == b"GBB1" and (trees, depth) == (100, 6) and len(enc) == 2000
    fmt, blob, trees, depth, row_format, enc = res[0]["gbdt_g32"]
    assert fmt == row_format == "g32" and blob[:4] == b"GBB1" and (trees, depth) == (100, 6) and len(enc) == 3200
    assert res[0]["mlp"][0] == res[0]["mlp"][4] == "w64"
