"""Communicator re-formation on membership change ("The RCCL communicator is
re-initialised on membership change"): heartbeats, generation proposals, a fresh process
group per generation, and X2 totals that keep every survivor's rows across a SIGKILL and a
rejoin.  CPU / gloo, real processes sharing a TCPStore hosted by the test."""
import datetime
import os
import signal
import socket
import time

import torch

from ccfd_demo_summit_amd.parallel.elastic import MemoryStore
from ccfd_demo_summit_amd.parallel.membership import Membership


class Clock:
    def __init__(self):
        self.t = 100.0

    def __call__(self):
        return self.t


def test_membership_generations_on_death_and_rejoin():
    store, clock = MemoryStore(), Clock()
    ms = [Membership(store, r, 3, ttl_s=1.0, grace_s=2.0, clock=clock) for r in range(3)]
    for m in ms:
        m.heartbeat()
    for m in ms:
        assert m.propose() is None                # live set == generation 0 (all ranks)
    assert ms[0].view() == (0, [0, 1, 2])
    # rank 1 stops heartbeating; after ttl the lowest live rank proposes {0, 2}
    for _ in range(3):
        clock.t += 0.5
        ms[0].heartbeat(); ms[2].heartbeat()
        ms[2].propose()                           # not the leader: never proposes
        ms[0].propose()
    assert ms[2].view() == (1, [0, 2])
    # a restarted rank 1 heartbeats again -> generation 2 includes it
    ms[1] = Membership(store, 1, 3, ttl_s=1.0, clock=clock)
    ms[1].heartbeat()
    clock.t += 0.1
    ms[0].heartbeat(); ms[2].heartbeat()
    assert ms[0].propose() == (2, [0, 1, 2])
    assert ms[1].view() == (2, [0, 1, 2])


def _member_proc(rank, world, port, phases):
    import torch.distributed as dist
    from ccfd_demo_summit_amd.parallel.membership import ElasticCounterReducer, ElasticGroup
    store = dist.TCPStore("127.0.0.1", port, is_master=False, timeout=datetime.timedelta(seconds=60))
    grp = ElasticGroup(store, rank, world, backend="gloo", ttl_s=1.0, timeout_s=10.0, grace_s=20.0)
    red = ElasticCounterReducer(grp, 2)
    done = set()
    while not store.check(["stop"]):
        if grp.tick():
            red.on_regroup()
        for ph in phases:
            if ph not in done and store.check([f"phase{ph}"]):
                red.submit(torch.tensor([10, 10 * (rank + 1)], dtype=torch.int64))
                done.add(ph)
        red.progress()
        t = red.totals.tolist()
        store.set(f"tot/{rank}", f"{grp.gen}|{','.join(map(str, grp.members))}|{t[0]},{t[1]}|{red.completed}")
        time.sleep(0.01)
    grp.close()


def _state(store, r):
    if not store.check([f"tot/{r}"]):
        return None
    gen, mem, tot, comp = store.get(f"tot/{r}").decode().split("|")
    return int(gen), [int(x) for x in mem.split(",") if x], [int(x) for x in tot.split(",")], int(comp)


def _wait(pred, timeout, what):
    t0 = time.time()
    while time.time() - t0 < timeout:
        if pred():
            return
        time.sleep(0.05)
    raise AssertionError(f"timed out waiting for {what}")


def test_sigkill_regroup_and_rejoin_keep_survivor_rows():
    import torch.distributed as dist
    import torch.multiprocessing as mp
    s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
    store = dist.TCPStore("127.0.0.1", port, 1, True, timeout=datetime.timedelta(seconds=60), wait_for_workers=False)
    ctx = mp.get_context("spawn")
    ps = {r: ctx.Process(target=_member_proc, args=(r, 3, port, ("A", "B", "C"))) for r in range(3)}
    for p in ps.values():
        p.start()
    rejoin = None
    try:
        # phase A: every rank contributes [10, 10 (r+1)] -> [30, 60] everywhere
        store.set("phaseA", "1")
        _wait(lambda: all((st := _state(store, r)) and st[2] == [30, 60] for r in range(3)), 120, "phase A totals")
        # SIGKILL rank 1, and let the survivors contribute while their group is broken
        os.kill(ps[1].pid, signal.SIGKILL)        # exact PID of our own child
        ps[1].join(10)
        store.set("phaseB", "1")
        _wait(lambda: all((st := _state(store, r)) and st[1] == [0, 2] for r in (0, 2)), 60, "regroup to [0, 2]")
        # nothing a survivor counted is lost: A + survivors' B = [30+20, 60+10+30]
        _wait(lambda: all(_state(store, r)[2] == [50, 100] for r in (0, 2)), 60, "phase B totals")
        gen_b = _state(store, 0)[0]
        assert gen_b >= 1
        # a restarted rank 1 rejoins: a new generation with all three members
        rejoin = ctx.Process(target=_member_proc, args=(1, 3, port, ("C",)))
        rejoin.start()
        _wait(lambda: all((st := _state(store, r)) and st[1] == [0, 1, 2] and st[0] > gen_b for r in range(3)),
              120, "rejoin generation")
        store.set("phaseC", "1")
        _wait(lambda: all(_state(store, r)[2] == [80, 160] for r in (0, 2)), 60, "phase C totals (survivors)")
        _wait(lambda: _state(store, 1)[2] == [30, 60], 60, "phase C totals (rejoined rank)")
        assert _state(store, 1)[3] > 0
    finally:
        store.set("stop", "1")
        for p in list(ps.values()) + ([rejoin] if rejoin is not None else []):
            p.join(20)
            if p.is_alive():
                p.kill()
