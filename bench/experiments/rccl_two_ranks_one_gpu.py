"""Can two ranks form an RCCL communicator on ONE GPU (the 1-GPU box is the only GPU a test can
get)?  Each rank all-reduces a tensor on cuda:0 through the `nccl` (RCCL) backend, then the
engine's X2 counter reduction (parallel.dp.CounterReducer) runs once.  Prints one JSON line per
rank; any error is printed and the rank exits non-zero.

Answer on the pool's 1-GPU MI355X box (round 5, `profiles/r5/rccl_two_ranks/out.log`): no --
RCCL 2.26.6 refuses at communicator init ("Duplicate GPU detected: rank 0 and rank 1 both on
CUDA device").  Multi-rank RCCL therefore first runs in the driver's 8-GPU scaling bench; the
rank logic is covered on gloo (tests/test_dist_cpu.py) and by the one-GPU gloo rehearsals.

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \\
        bench/experiments/rccl_two_ranks_one_gpu.py
"""
import json
import os
import sys
import time

import torch
import torch.distributed as dist


def main() -> int:
    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    t0 = time.time()
    try:
        dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
        x = torch.full((1 << 20,), float(rank + 1), device="cuda")
        dist.all_reduce(x)
        torch.cuda.synchronize()
        ok = bool((x == sum(range(1, world + 1))).all())
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
        from ccfd_demo_summit_amd.parallel import CounterReducer, DistContext
        ctx = DistContext(rank, world, 0, torch.device("cuda", 0), "nccl")
        red = CounterReducer(ctx, torch.device("cuda", 0))
        import numpy as np
        c = torch.zeros(64, dtype=torch.int64, device="cuda")
        c[0] = 10 * (rank + 1)
        red.submit(c, np.ones(256, np.int64))
        red.wait()
        g, _ = red.snapshot()
        print(json.dumps({"rank": rank, "world": world, "allreduce_ok": ok, "x2_counter": int(g[0]),
                          "x2_expected": 10 * sum(range(1, world + 1)), "s": round(time.time() - t0, 2)}), flush=True)
        dist.barrier()
        dist.destroy_process_group()
        return 0 if ok else 1
    except Exception as e:                                  # noqa: BLE001 -- the answer is the point
        print(json.dumps({"rank": rank, "error": repr(e)[:500]}), flush=True)
        return 2


if __name__ == "__main__":
    sys.exit(main())
