"""Data-parallel training at world size 2 on CPU (gloo): the reference trains on a
2-executor Spark cluster (deploy/frauddetection_cr.yaml:27,34-35).

* MLP / LR under DDP: every rank ends with bit-identical parameters (gradients all-reduced)
  and the loss falls;
* oblivious GBDT with all-reduced histograms: every rank grows the same ensemble, and it is
  the ensemble a single process grows on the union of the shards (float summation order
  aside)."""
import os
import socket

import numpy as np
import torch.multiprocessing as mp

from ccfd_demo_summit_amd.data import generate


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _data():
    X, y = generate(12000, seed=77, fraud_rate=0.05)
    return X, y


def _worker(rank, world, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    from ccfd_demo_summit_amd.train.trainer import (TrainConfig, _quantile_borders, train_logistic, train_mlp,
                                                    train_oblivious_gbdt)
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        X, y = _data()               # every rank passes all rows and trains on rows rank::world
        cfg = TrainConfig(epochs=2, batch=512, device="cpu", bf16=False, graph=False, seed=3)
        mlp, info = train_mlp(X, y, cfg)
        lr, info_lr = train_logistic(X, y, cfg)
        gb, info_gb = train_oblivious_gbdt(X, y, n_trees=8, depth=4, device="cpu",
                                           borders=_quantile_borders(X, 32))
        q.put((rank, [np.asarray(a) for a in (mlp.W1, mlp.W2, mlp.w3, lr.w)], info["steps"], info["final_loss"],
               gb.feat.copy(), gb.thr.copy(), gb.leaves.copy(), gb.base, info_gb))
    finally:
        dist.destroy_process_group()


def test_ddp_and_gbdt_data_parallel_world2():
    from ccfd_demo_summit_amd.train.trainer import _quantile_borders, train_oblivious_gbdt
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=240) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (_, p0, steps0, loss0, f0, t0, l0, b0, i0), (_, p1, steps1, loss1, f1, t1, l1, b1, i1) = res
    # DDP: identical parameters on both ranks, each rank stepped over its half of the rows
    for a, b in zip(p0, p1):
        np.testing.assert_array_equal(a, b)
    assert steps0 == steps1 == 2 * int(np.ceil(6000 / 512))
    assert np.isfinite(loss0) and np.isfinite(loss1)
    # GBDT: same ensemble on both ranks ...
    np.testing.assert_array_equal(f0, f1)
    np.testing.assert_array_equal(t0, t1)
    np.testing.assert_array_equal(l0, l1)
    assert b0 == b1 and i0["world"] == 2
    # ... and the one a single process grows on all rows
    X, y = _data()
    ref, info = train_oblivious_gbdt(X, y, n_trees=8, depth=4, device="cpu", borders=_quantile_borders(X, 32))
    np.testing.assert_array_equal(f0, ref.feat)
    np.testing.assert_array_equal(t0, ref.thr)
    np.testing.assert_allclose(l0, ref.leaves, rtol=1e-4, atol=1e-6)
    assert abs(b0 - ref.base) < 1e-9
    assert abs(i0["train_logloss"] - info["train_logloss"]) < 1e-5
