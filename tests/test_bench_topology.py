"""bench.py refuses to report an N-GPU number from a topology that is not N ranks on N
distinct GPUs over RCCL (VERDICT r1 "Next #1"); --rehearsal runs it anyway but labels it.
CPU: gloo, world 2, with synthetic device identities."""
import os
import socket
import sys
from pathlib import Path
from types import SimpleNamespace

import pytest
import torch.multiprocessing as mp

ROOT = Path(__file__).resolve().parents[1]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, gpus, same_pci, rehearsal, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, str(ROOT))
    import torch.distributed as dist
    import bench
    from ccfd_demo_summit_amd.parallel import init_distributed
    ctx = init_distributed(backend="gloo")
    args = SimpleNamespace(gpus=gpus, rehearsal=rehearsal)
    ident = {"rank": rank, "host": "node0", "device": 0,
             "pci": "0000:05:00" if same_pci else f"0000:{5 + rank:02x}:00", "name": "x"}
    try:
        idents, problems = bench._verify_topology(args, ctx, ident)
        q.put((rank, "ok", problems, [d["pci"] for d in idents]))
    except SystemExit as e:
        q.put((rank, "exit", e.code, None))
    finally:
        dist.destroy_process_group()


def _run(world, gpus, same_pci, rehearsal):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, gpus, same_pci, rehearsal, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    return res


def test_gloo_backend_refused_without_rehearsal():
    # world 2 over gloo (not RCCL) -> every rank exits non-zero
    res = _run(2, 2, same_pci=False, rehearsal=False)
    assert [r[1] for r in res] == ["exit", "exit"] and all(r[2] == 3 for r in res)


def test_rehearsal_labels_every_problem():
    res = _run(2, 4, same_pci=True, rehearsal=True)
    for rank, kind, problems, pcis in res:
        assert kind == "ok"
        text = " ".join(problems)
        assert "WORLD_SIZE=2" in text and "gloo" in text and "share GPU 0000:05:00" in text
        assert pcis == ["0000:05:00", "0000:05:00"]


def test_single_rank_mismatch_refused():
    sys.path.insert(0, str(ROOT))
    import bench
    from ccfd_demo_summit_amd.parallel.dp import DistContext
    ctx = DistContext()
    with pytest.raises(SystemExit):
        bench._verify_topology(SimpleNamespace(gpus=8, rehearsal=False), ctx,
                               {"rank": 0, "host": "h", "device": 0, "pci": "0000:05:00", "name": "x"})
    idents, problems = bench._verify_topology(SimpleNamespace(gpus=1, rehearsal=False), ctx,
                                              {"rank": 0, "host": "h", "device": 0, "pci": "p", "name": "x"})
    assert problems == [] and idents[0]["pci"] == "p"


def test_e2e_refuses_isolated_stacks_at_n_gt_1():
    """bench/e2e.py builds a private broker + KIE per rank: at WORLD_SIZE > 1 that is N isolated
    stacks, not config 5 -- refused without --allow-isolated, and labelled when allowed."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, WORLD_SIZE="2", RANK="0")
    r = subprocess.run([sys.executable, os.path.join(root, "bench", "e2e.py"), "--seconds", "1"],
                       capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode != 0 and "deploy_topology.py" in r.stderr, r.stderr[-500:]
    src = open(os.path.join(root, "bench", "e2e.py")).read()
    assert '"isolated-per-rank"' in src and '"topology"' in src
