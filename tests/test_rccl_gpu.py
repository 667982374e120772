"""The X2/X1 code path over the real RCCL backend (one rank: RCCL runs its kernels for a
1-rank communicator too), so the async all-reduce / is_completed / side-stream ordering and
the async hot-swap broadcast are exercised on the GPU, not only over gloo."""
import os
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


class _Ctx:
    """DistContext that reports itself initialised with world == 1 (forces the collective path)."""

    def __init__(self, device):
        self.rank, self.world, self.local_rank, self.device, self.backend = 0, 1, 0, device, "nccl"

    @property
    def initialized(self):
        return True


@pytest.fixture(scope="module")
def nccl():
    import torch.distributed as dist
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    yield dev
    dist.destroy_process_group()


def test_async_counter_allreduce_over_rccl(nccl):
    from ccfd_demo_summit_amd.parallel import CounterReducer, EpochPipeline, x_group
    from ccfd_demo_summit_amd.engine import PartitionLog, StreamEngine
    from ccfd_demo_summit_amd.data import generate
    from ccfd_demo_summit_amd.models import build_model
    from ccfd_demo_summit_amd.ops.kernels import DeviceModel
    ctx = _Ctx(nccl)
    X, _ = generate(50_000, seed=4)
    m = build_model("mlp", seed=3, X_ref=X[:10000], calibrate_rate=0.05)
    eng = StreamEngine(DeviceModel(m, nccl), batch=2048, depth=8, input_mode="zerocopy", exec_mode="persistent")
    log = PartitionLog.from_arrays(X)
    eng.add_log(0, log)
    red = CounterReducer(ctx, nccl, group=None)
    ep = EpochPipeline(eng, red)
    total = deferred = 0
    for k in range(20):
        eng.pump(5, drain=(k % 5 == 4))
        total += 5 * 2048
        if not ep.tick(progress=lambda: eng.run(0, 0), block=(k % 2 == 0)):
            deferred += 1
    eng.pump(0, drain=True)
    ep.finish(progress=lambda: eng.run(0, 0))
    c, _ = red.snapshot()
    assert c[0] == total and c[1] + c[2] == total
    assert not red.busy()
    eng.close()
    log.free()


def test_async_hot_swap_broadcast_over_rccl(nccl):
    from ccfd_demo_summit_amd.models import build_model
    from ccfd_demo_summit_amd.ops.kernels import DeviceModel
    from ccfd_demo_summit_amd.parallel.hotswap import HotSwap

    class Eng:
        wire = False

        def __init__(self):
            self.dm = DeviceModel(build_model("mlp", seed=1), nccl)
            self.swapped = []

        def swap_model(self, dm):
            self.dm = dm
            self.swapped.append(bytes(dm.blob.cpu().numpy()))

    eng = Eng()
    hs = HotSwap(_Ctx(nccl), eng)
    new = build_model("mlp", seed=2)
    hs.offer(new)
    v = hs.contribute()
    assert v[0] == 1 and v[1] == len(new.pack())
    hdr = torch.from_numpy(v).to(nccl)
    import torch.distributed as dist
    dist.all_reduce(hdr)                     # what the X2 reduce carries
    hs.on_reduced(hdr.cpu().numpy())
    assert hs.poll(block=True)
    assert hs.version == 1 and eng.swapped == [new.pack()]
    assert hs.tick() is False                # nothing offered: header all-reduce only


def test_elastic_group_rebuilds_rccl_communicator(nccl):
    """parallel/membership.py over RCCL: a 1-member ProcessGroupNCCL per generation on a
    PrefixStore (independent of the default group), async all-reduce of GPU counters polled
    to completion; a forced new generation aborts the old communicator and builds a new one."""
    import datetime
    import time
    import torch.distributed as dist
    from ccfd_demo_summit_amd.parallel.membership import ElasticCounterReducer, ElasticGroup
    s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
    store = dist.TCPStore("127.0.0.1", port, 1, True, timeout=datetime.timedelta(seconds=30), wait_for_workers=False)
    grp = ElasticGroup(store, 0, 1, backend="nccl", device=nccl, ttl_s=1.0)
    red = ElasticCounterReducer(grp, 4)
    assert grp.tick() and grp.member and grp.members == [0]
    red.submit(torch.tensor([1, 2, 3, 4], device=nccl))
    t0 = time.time()
    while red.completed < 2 and time.time() - t0 < 30:
        red.progress()
    assert red.totals.tolist() == [1, 2, 3, 4]
    # a new generation (e.g. a rank rejoined) -> abort + rebuild, nothing local is lost
    gen0 = grp.gen
    red.submit(torch.tensor([10, 0, 0, 0], device=nccl))
    red.progress()
    store.set("ccfd/mem/gen", f"{gen0 + 1}:0")
    assert grp.tick() and grp.gen == gen0 + 1
    red.on_regroup()
    t0 = time.time()
    while red.totals[0].item() < 11 and time.time() - t0 < 30:
        red.progress()
    assert red.totals.tolist() == [11, 2, 3, 4]
    grp.close()
