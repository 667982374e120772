#!/usr/bin/env python3
"""Which RCCL collectives launch a device kernel on a ONE-rank communicator?

Run under ``rocprofv3 --kernel-trace --stats`` on one GPU.  Expected (RCCL follows NCCL's
one-rank shortcut): an in-place SUM all-reduce -- the X2 counter reduction -- launches
nothing; ncclAvg / PreMulSum launch ``OneRankReduce``.  This decides how the X2 overlap
trace on a one-GPU box can show an RCCL kernel next to the persistent scoring kernel
(profiles/r3/x2_overlap/README.md).
"""
import os
import sys

import torch
import torch.distributed as dist

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29541")
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
out = {}
for name, dtype, op in (("sum_i64", torch.int64, dist.ReduceOp.SUM), ("avg_i64", torch.int64, dist.ReduceOp.AVG),
                        ("avg_f32", torch.float32, dist.ReduceOp.AVG), ("sum_f32", torch.float32, dist.ReduceOp.SUM)):
    t = torch.arange(324, dtype=dtype, device=dev)
    ref = t.clone()
    try:
        for _ in range(5):
            dist.all_reduce(t, op=op)
        torch.cuda.synchronize()
        out[name] = "ok" if torch.equal(t, ref) else "changed"
    except Exception as e:                 # an op this RCCL / dtype does not support
        out[name] = f"error: {e}"[:200]
g = torch.empty(324 * 1, dtype=torch.int64, device=dev)
dist.all_gather_into_tensor(g, torch.arange(324, dtype=torch.int64, device=dev))
torch.cuda.synchronize()
out["all_gather_i64"] = "ok"
print(out, flush=True)
dist.destroy_process_group()
sys.exit(0)
