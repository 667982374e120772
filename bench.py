#!/usr/bin/env python3
"""Headline benchmark: streaming fraud scoring, transactions/s (whole node) + p50 latency.

BASELINE.json metric "transactions/sec (whole node) + p50 scoring latency at 1/2/4/8
MI355X", config 2/3: 3-layer MLP 30->128->64->1, bf16 MFMA, micro-batch 4096,
data-parallel stream shard (one process per GPU, RCCL over xGMI).

One *step* per rank = ``--batches-per-step`` micro-batches of ``--batch`` transactions
consumed from that rank's partition logs (pinned host memory, pre-filled by the synthetic
producer = the reference's producer replaying creditcard.csv onto the topic), each:
H2D (or zero-copy) -> fused HIP kernel (normalize + MLP + sigmoid + FRAUD_THRESHOLD route +
device counters + amount histogram) -> proba/route into pinned host slots -> completion ->
flagged transactions pushed to the hand-off ring, which the step drains (router ->
fraud-process hand-off); then the epoch's device counters + latency histogram are
all-reduced over RCCL on a side stream (X2/X3), overlapped with the next step.

    python bench.py                      # 1 GPU, defaults finish in well under a minute
    torchrun --nproc-per-node 8 bench.py --gpus 8 --steps 100 --warmup 10

Rank 0 prints ONE JSON line; ``value`` = total rows scored by all ranks / max-over-ranks
time of the K timed steps.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

METRIC = "transactions/sec (whole node) + p50 scoring latency at 1/2/4/8 MI355X"


def parse_args(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--model", default="mlp", choices=["mlp", "lr", "gbdt"])
    ap.add_argument("--batch", type=int, default=4096, help="micro-batch rows")
    ap.add_argument("--batches-per-step", type=int, default=256)
    ap.add_argument("--depth", type=int, default=32, help="micro-batches in flight per GPU")
    ap.add_argument("--streams", type=int, default=4)
    ap.add_argument("--input-mode", default="zerocopy", choices=["dma", "zerocopy"])
    ap.add_argument("--output-mode", default="zerocopy", choices=["zerocopy", "dma"])
    ap.add_argument("--exec-mode", default="auto", choices=["auto", "launch", "persistent"],
                    help="auto = persistent kernel for mlp/lr with zero-copy in/out, coalesced launches "
                         "otherwise (profiles/r1/persist_sweep.txt)")
    ap.add_argument("--persist-grid", type=int, default=0, help="persistent workgroups (0 = engine default 128)")
    ap.add_argument("--coalesce", type=int, default=8,
                    help="launch mode: ready micro-batches per kernel launch (each keeps its own completion)")
    ap.add_argument("--wire", default="auto", choices=["auto", "f32", "w64"],
                    help="partition-log row format: 30 x f32 (120 B) or W64 (64 B: bf16 V1..V28, "
                         "f32 Time/Amount; contracts/transaction.py). auto = w64 for mlp/lr "
                         "(the zero-copy path is PCIe-bound; profiles/r1/wire_sweep.txt), f32 for gbdt")
    ap.add_argument("--log-rows", type=int, default=1 << 22, help="rows per rank (pinned partition logs)")
    ap.add_argument("--partitions-per-rank", type=int, default=2)
    ap.add_argument("--threshold", type=float, default=0.5)
    ap.add_argument("--gbdt-trees", type=int, default=100)
    ap.add_argument("--gbdt-depth", type=int, default=6)
    ap.add_argument("--x2-every", type=int, default=8,
                    help="steps between X2 counter all-reduces (8 x ~1.3 ms = the >= 10 ms reduction "
                         "period of SURVEY.md 2.5); a step count, so every rank issues the same collectives")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--no-unloaded-probe", action="store_true")
    ap.add_argument("--out", default=None, help="also write the JSON line to this file")
    return ap.parse_args(argv)


def baseline_value():
    """Config-1 reference-topology number measured by us, or None."""
    p = ROOT / "bench" / "baseline_measured.json"
    if p.exists():
        try:
            return float(json.loads(p.read_text())["cpu_lr_batch1_seldon_rest_tx_per_s"])
        except Exception:
            return None
    return None


def main(argv=None):
    args = parse_args(argv)
    if args.wire == "auto":
        args.wire = "w64" if args.model in ("mlp", "lr") else "f32"
    import torch
    from ccfd_demo_summit_amd.data import FRAUD_RATE, generate
    from ccfd_demo_summit_amd.engine import PartitionLog, StreamEngine
    from ccfd_demo_summit_amd.models import build_model
    from ccfd_demo_summit_amd.ops.kernels import DeviceModel
    from ccfd_demo_summit_amd.parallel import (CounterReducer, EpochPipeline, all_max, assign_partitions,
                                               barrier, broadcast_blob, hist_quantile, init_distributed)

    ctx = init_distributed()
    if ctx.world != args.gpus:
        if ctx.rank == 0:
            print(f"[bench] note: --gpus {args.gpus} but WORLD_SIZE={ctx.world}; using WORLD_SIZE",
                  file=sys.stderr)
    if not torch.cuda.is_available():
        raise SystemExit("bench.py needs a GPU (MI355X)")
    dev = ctx.device
    W = ctx.world
    from ccfd_demo_summit_amd.utils.numa import bind_to_gpu
    numa_node = bind_to_gpu(dev.index)     # pinned logs + host threads on the GPU's socket

    # ---- model: rank 0 builds (random init of the named architecture; normaliser fitted and
    # output bias calibrated on a synthetic sample so ~0.17 % of traffic routes to the fraud
    # process, like the dataset prior), X1 broadcast over RCCL to every rank.
    if ctx.rank == 0:
        Xcal, _ = generate(200_000, seed=args.seed + 999)
        model = build_model(args.model, seed=args.seed, X_ref=Xcal, calibrate_rate=FRAUD_RATE,
                            threshold=args.threshold, gbdt_trees=args.gbdt_trees, gbdt_depth=args.gbdt_depth)
        packed = model.pack(wire=True) if args.wire == "w64" else model.pack()
        blob = torch.from_numpy(np.frombuffer(packed, np.uint8).copy()).to(dev)
    else:
        blob = None
    blob = broadcast_blob(ctx, blob)
    trees = args.gbdt_trees if args.model == "gbdt" else 0
    depth_t = args.gbdt_depth if args.model == "gbdt" else 0
    dm = DeviceModel.from_blob(args.model, blob, trees, depth_t, wire=args.wire == "w64")
    exec_mode = args.exec_mode
    if exec_mode == "auto":
        # measured on MI355X (profiles/r1/persist_sweep.txt): the persistent kernel with a
        # parallel doorbell and 512-row work items reaches 0.82e9 tx/s at p50 147 us, above
        # coalesced launches (0.75e9 at 166 us); GBDT and DMA paths use launches
        zc = args.input_mode == "zerocopy" and args.output_mode == "zerocopy"
        exec_mode = "persistent" if args.model in ("mlp", "lr") and zc else "launch"

    # ---- this rank's partitions of topic odh-demo (p % W == rank), pre-filled logs
    n_parts = args.partitions_per_rank * W
    my_parts = assign_partitions(n_parts, ctx.rank, W)
    rows_per_part = max(args.batch * 4, args.log_rows // len(my_parts))
    logs = []
    eng = StreamEngine(dm, batch=args.batch, depth=args.depth, streams=args.streams,
                       input_mode=args.input_mode, output_mode=args.output_mode,
                       threshold=args.threshold, device=dev.index, exec_mode=exec_mode,
                       persist_grid=args.persist_grid, coalesce=args.coalesce)
    for p in my_parts:
        log = PartitionLog(rows_per_part, wire=args.wire == "w64")
        if log.wire:
            Xp, _ = generate(rows_per_part, seed=args.seed * 7919 + p)
            log.write_rows(0, Xp)           # ingest-side encoding, outside the timed region
            del Xp
        else:
            generate(rows_per_part, seed=args.seed * 7919 + p, out=log.feats.array)
        log.ids.array[:] = np.arange(rows_per_part, dtype=np.uint64) + np.uint64(p) * np.uint64(1 << 40)
        log.customer.array[:] = np.random.default_rng(p).integers(0, 1_000_000, rows_per_part, dtype=np.uint32)
        eng.add_log(p, log)
        logs.append(log)

    reducer = CounterReducer(ctx, dev, priority=0)
    epochs = EpochPipeline(eng, reducer)
    flagged_total = 0
    x2_s = [0.0]

    nstep = [0]

    def step(drain: bool):
        nonlocal flagged_total
        eng.pump(args.batches_per_step, drain=drain)
        # router hand-off of fraud-routed transactions (transaction.outgoing{type=fraud})
        flagged_total += len(eng.drain_flagged())
        nstep[0] += 1
        if nstep[0] % max(1, args.x2_every):
            return
        # X2/X3: flip the counter epoch; the previously closed epoch (all of whose batches
        # have completed by now) is all-reduced over RCCL on the side stream
        tx = time.perf_counter()
        epochs.tick(progress=lambda: eng.run(0, 0))   # (retire finished batches if it must wait)
        x2_s[0] += time.perf_counter() - tx

    for _ in range(args.warmup):
        step(drain=False)
    eng.pump(0, drain=True)
    epochs.finish()
    eng.reset_stats()
    c0 = reducer.snapshot()[0]
    rows0, fraud0 = int(c0[0]), int(c0[1])
    eng.drain_flagged()          # warmup hand-offs are not part of the timed run
    flagged_total = 0
    x2_s[0] = 0.0
    nstep[0] = 0
    barrier(ctx)
    torch.cuda.synchronize(dev)

    t0 = time.perf_counter()
    for k in range(args.steps):
        step(drain=(k == args.steps - 1))
    epochs.finish()
    torch.cuda.synchronize(dev)
    barrier(ctx)
    t1 = time.perf_counter()
    elapsed = all_max(ctx, t1 - t0)

    # latency: per-rank histogram of the timed batches, merged over ranks (X3)
    st_final = eng.pump(0, drain=True)
    lat_local = st_final.lat_hist.astype(np.int64)
    lat_t = torch.from_numpy(lat_local).to(dev)
    if ctx.initialized:
        import torch.distributed as dist
        dist.all_reduce(lat_t)
    lat = lat_t.cpu().numpy()
    counters, _ = reducer.snapshot()
    total_rows = int(counters[0] - rows0)
    expected = args.steps * args.batches_per_step * args.batch * W
    p50_us = hist_quantile(lat, 0.50) / 1e3
    p99_us = hist_quantile(lat, 0.99) / 1e3

    # unloaded latency probe (not timed): one micro-batch at a time, depth 1
    p50_unloaded = None
    if not args.no_unloaded_probe:
        probe = StreamEngine(dm, batch=args.batch, depth=1, streams=1, input_mode=args.input_mode,
                             output_mode=args.output_mode, threshold=args.threshold, device=dev.index,
                             exec_mode=exec_mode)
        probe.add_log(my_parts[0], logs[0])
        probe.pump(20, drain=True)
        probe.reset_stats()
        sp = probe.pump(200, drain=True)
        p50_unloaded = sp.p50_us
        probe.close()

    value = total_rows / elapsed
    base = baseline_value()
    out = {
        "metric": METRIC,
        "value": round(value, 1),
        "unit": "tx/s",
        "n_gpus": W,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": (round(value / base, 1) if base else None),
        "dtype": "bf16" if args.model == "mlp" else "fp32",
        "data": ("synthetic creditcard-shaped transactions (30 features; log rows "
                 + ("W64: bf16 V1..V28 + f32 Time/Amount, 64 B" if args.wire == "w64" else "30 x f32, 120 B")
                 + ") replayed from pinned partition logs; random-init weights, normaliser fitted + "
                 "output bias calibrated to the 0.172% fraud prior on a synthetic sample"),
        "config": {"model": {"mlp": "mlp_30_128_64_1", "lr": "logreg_30",
                             "gbdt": f"oblivious_gbdt_{args.gbdt_trees}x{args.gbdt_depth}"}[args.model],
                   "global_batch": args.batch * W, "seq_len": 1, "micro_batch": args.batch,
                   "parallelism": f"dp{W}", "input_mode": args.input_mode,
                   "output_mode": args.output_mode, "exec_mode": exec_mode, "depth": args.depth,
                   "wire": args.wire, "coalesce": args.coalesce,
                   "streams": args.streams,
                   "batches_per_step": args.batches_per_step, "x2_every_steps": args.x2_every,
                   "numa_node_rank0": numa_node},
        "p50_latency_us": round(p50_us, 2),
        "p99_latency_us": round(p99_us, 2),
        "p50_latency_us_unloaded": None if p50_unloaded is None else round(p50_unloaded, 2),
        # engine host-thread time per timed micro-batch (cumulative since reset_stats)
        "host_us_per_batch": {k: round(v * 1e6 / (args.steps * args.batches_per_step), 3) for k, v in
                              (("submit", st_final.host_submit_s), ("wait", st_final.host_wait_s),
                               ("complete", st_final.host_complete_s))},
        # host time per step spent in the X2 tick (epoch flip + side-stream all-reduce issue)
        "host_us_per_step_x2": round(x2_s[0] * 1e6 / args.steps, 2),
        "step_us_per_batch": round(elapsed * 1e6 / (args.steps * args.batches_per_step), 3),
        # K7: per-micro-batch execution window on the GPU's own clock (rank 0)
        "device_exec_us_mean": round(st_final.dev_exec_mean_us, 2),
        "device_exec_us_p50": round(hist_quantile(st_final.dev_hist.astype(np.int64), 0.5) / 1e3, 2)
        if st_final.dev_batches else None,
        "rows_scored": total_rows,
        "rows_expected": expected,
        "fraud_routed": int(counters[1]) - fraud0,
        "flagged_handed_off_rank0": flagged_total,
    }
    if total_rows != expected and ctx.rank == 0:
        print(f"[bench] WARNING: counted {total_rows} rows, expected {expected}", file=sys.stderr)
    if ctx.rank == 0:
        line = json.dumps(out)
        print(line, flush=True)
        if args.out:
            Path(args.out).write_text(line + "\n")
    eng.close()
    if ctx.initialized:
        import torch.distributed as dist
        barrier(ctx)
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
