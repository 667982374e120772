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
    python bench.py --gpus 8             # spawns 8 local ranks (torch.distributed.run child)
    torchrun --nproc-per-node 8 bench.py --gpus 8 --steps 100 --warmup 10   # same, driver-style

Rank 0 prints ONE JSON line; ``value`` = total rows scored by all ranks / max-over-ranks
time of the K timed steps.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
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
    ap.add_argument("--batch", type=int, default=None,
                    help="micro-batch rows (default: the BASELINE config's -- 4096 for mlp/lr, 65536 for gbdt)")
    ap.add_argument("--batches-per-step", type=int, default=256)
    ap.add_argument("--depth", type=int, default=None,
                    help="micro-batches in flight per GPU (default 12 for mlp/lr = p50 53 us at the "
                         "PCIe-bound rate, profiles/r2/persist_full_item/; 3 for gbdt = 1.67e9 tx/s at "
                         "p50 107 us with 65536-row batches, profiles/r2/persist_full_item/g32_inflight_ab.jsonl; "
                         "--batch 16384 --depth 8 gives p50 74 us at 1.64e9, "
                         "profiles/r2/gbdt_g32_operating_curve.jsonl)")
    ap.add_argument("--streams", type=int, default=4)
    ap.add_argument("--input-mode", default="zerocopy", choices=["dma", "zerocopy"])
    ap.add_argument("--output-mode", default="zerocopy", choices=["zerocopy", "dma"])
    ap.add_argument("--exec-mode", default="auto", choices=["auto", "launch", "persistent"],
                    help="auto = persistent kernel for mlp/lr and for gbdt on G32 rows with zero-copy "
                         "in/out, launches otherwise (profiles/r1/persist_sweep.txt, profiles/r2/)")
    ap.add_argument("--trace", default=None,
                    help="rank 0: write a Chrome / Perfetto timeline of the last 65536 timed micro-batches "
                         "(per-batch stage trace: queued, in flight, device, hand-off)")
    ap.add_argument("--persist-grid", type=int, default=0, help="persistent workgroups (0 = engine default: 64 for W64 rows, 216 for G20, 128 otherwise)")
    ap.add_argument("--coalesce", type=int, default=8,
                    help="launch mode: ready micro-batches per kernel launch (each keeps its own completion)")
    ap.add_argument("--wire", default="auto", choices=["auto", "f32", "w64", "g32", "g20"],
                    help="partition-log row format: 30 x f32 (120 B), W64 (64 B: bf16 V1..V28, "
                         "f32 Time/Amount), G32 (32 B, GBDT: u8 bin per feature against the "
                         "ensemble's split table -- exact; contracts/transaction.py) or G20 (20 B: the "
                         "same bins, 5 bits each, for <= 31 thresholds a feature). auto = w64 for "
                         "mlp/lr (the zero-copy path is PCIe-bound; profiles/r1/wire_sweep.txt), g20 for "
                         "gbdt (widening to g32 / f32 when the ensemble's bin table needs it)")
    ap.add_argument("--log-rows", type=int, default=1 << 22, help="rows per rank (pinned partition logs)")
    ap.add_argument("--partitions-per-rank", type=int, default=2)
    ap.add_argument("--flag-capacity", type=int, default=1 << 23,
                    help="flagged (fraud-route) hand-off ring, records; sized so a step never "
                         "back-pressures on the step-end drain (a full ring stalls scoring, never drops)")
    ap.add_argument("--threshold", type=float, default=0.5)
    ap.add_argument("--gbdt-trees", type=int, default=100)
    ap.add_argument("--gbdt-depth", type=int, default=6)
    ap.add_argument("--x2-every", type=int, default=0,
                    help="steps between X2 counter all-reduces (SURVEY.md 2.5: >= 10 ms period); a step "
                         "count, so every rank issues the same collectives.  0 = derive from "
                         "--x2-period-ms and the calibrated step time")
    ap.add_argument("--x2-period-ms", type=float, default=10.0,
                    help="target X2 all-reduce period; --x2-every is derived from the calibrated step "
                         "time when --x2-every is 0 (default)")
    ap.add_argument("--min-timed-s", type=float, default=5.0,
                    help="sustained measurement: after warmup, --batches-per-step is raised (same value "
                         "on every rank) so that the K timed steps last at least this long (5 s: long "
                         "enough for an external utilisation sampler to see the load)")
    ap.add_argument("--watchdog-s", type=float, default=120.0,
                    help="exit non-zero with a per-rank diagnostic when no step completes for this long "
                         "(a wedged collective / doorbell; 0 = off)")
    ap.add_argument("--pg-timeout-s", type=float, default=180.0,
                    help="process-group (RCCL) collective timeout")
    ap.add_argument("--host-probe-s", type=float, default=0.3,
                    help="CPU-side streaming-read probe of each rank's NUMA node DRAM, all ranks at once "
                         "(predicts the host ceiling of N zero-copy ranks; 0 = off)")
    ap.add_argument("--encode-probe-rows", type=int, default=1 << 20,
                    help="rows for the untimed host row-encoder cost probe (W64 / G20 / G32 ingest "
                         "encoding done outside the timed region; 0 = off)")
    ap.add_argument("--rehearsal", action="store_true",
                    help="allow a rehearsal topology (WORLD_SIZE != --gpus, gloo collectives, several "
                         "ranks per GPU); the JSON line is then labelled rehearsal and must not be "
                         "quoted as an N-GPU number")
    ap.add_argument("--probe-ms", type=float, default=200.0,
                    help="per-rank zero-copy H2D bandwidth probe, all ranks concurrently (0 = off)")
    ap.add_argument("--precision-rows", type=int, default=1 << 20,
                    help="rows scored through the device kernel and compared with the fp32 oracle")
    ap.add_argument("--no-f32-probe", action="store_true",
                    help="skip the secondary f32-wire throughput run (W64 headline only)")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--no-unloaded-probe", action="store_true")
    ap.add_argument("--diagnostic", action="store_true",
                    help="allow diagnostic environment variables (utils/benchenv.py: an A/B library, fault "
                         "injection, launch serialisation, ...); the line is then labelled diagnostic and "
                         "must not be quoted as a headline")
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


def _fail(msg: str) -> None:
    print(f"[bench] FATAL: {msg}", file=sys.stderr, flush=True)
    raise SystemExit(3)


def _device_ident(ctx, dev) -> dict:
    import socket
    import torch
    p = torch.cuda.get_device_properties(dev.index)
    return {"rank": ctx.rank, "host": socket.gethostname(), "device": dev.index,
            "pci": f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}", "name": p.name}


def _verify_topology(args, ctx, ident: dict):
    """An N-GPU number must come from N ranks, one per distinct GPU, over RCCL.  Returns
    (per-rank device identities, problems); exits non-zero on any problem unless
    --rehearsal (then the line is labelled a rehearsal)."""
    problems = []
    if ctx.world != args.gpus:
        problems.append(f"--gpus {args.gpus} but WORLD_SIZE={ctx.world}")
    if ctx.world > 1 and ctx.backend != "nccl":
        problems.append(f"backend {ctx.backend!r} (an N>1 run must use nccl = RCCL over xGMI)")
    if os.environ.get("CCFD_DEVICE_MODULO") == "1" and ctx.world > 1:
        problems.append("CCFD_DEVICE_MODULO=1 maps several ranks onto one GPU")
    idents = [ident]
    if ctx.initialized:
        import torch.distributed as dist
        idents = [None] * ctx.world
        dist.all_gather_object(idents, ident)
        seen = {}
        for d in idents:
            key = (d["host"], d["pci"])
            if key in seen:
                problems.append(f"ranks {seen[key]} and {d['rank']} share GPU {d['pci']} on {d['host']}")
            seen.setdefault(key, d["rank"])
        if dist.get_world_size() != ctx.world:
            problems.append(f"process group size {dist.get_world_size()} != WORLD_SIZE {ctx.world}")
    if problems and not args.rehearsal:
        for m in problems:
            if ctx.rank == 0:
                print(f"[bench] topology check failed: {m}", file=sys.stderr)
        _fail("refusing to report an N-GPU number from this topology (use --rehearsal to run anyway)")
    return idents, problems


def _h2d_probe(lib_, ms: float, mb: int = 256) -> float:
    """Zero-copy kernel read bandwidth from this rank's pinned host memory (GB/s), run for
    ~``ms``: the better of 16-byte and 4-byte lanes (the link gives ~57.5 GB/s to 4-byte
    lanes and ~55.5 to 16-byte ones, profiles/r3/load_width/), so the reported ceiling is
    the link's, not one load width's.  All ranks run it at once, so host-DRAM and
    PCIe-root contention between ranks shows up here."""
    import ctypes as C
    import torch
    from ccfd_demo_summit_amd.engine import PinnedArray
    L = lib_()
    L.ccfd_bw_probe_width.argtypes = [C.c_void_p, C.c_size_t, C.c_int, C.c_int, C.c_int, C.c_void_p]
    L.ccfd_bw_probe_width.restype = C.c_double
    nbytes = mb << 20
    host = PinnedArray(nbytes // 4, "float32")
    host.array[:] = 1.0
    scratch = torch.empty(1 << 16, dtype=torch.uint8, device="cuda")
    try:
        best = 0.0
        for width in (16, 4):
            one = L.ccfd_bw_probe_width(C.c_void_p(host.ptr), nbytes, width, 2048, 1, C.c_void_p(scratch.data_ptr()))
            iters = max(1, int(ms / 2e3 * one * 1e9 / nbytes)) if one > 0 else 1
            best = max(best, float(L.ccfd_bw_probe_width(C.c_void_p(host.ptr), nbytes, width, 2048, iters,
                                                         C.c_void_p(scratch.data_ptr()))))
        return best
    finally:
        host.free()


def _host_read_probe(lib_, seconds: float, threads: int = 0, mb: int = 2048):
    """CPU streaming-read GB/s of this rank's NUMA node (the process is already bound to its
    GPU's node): the DRAM side of the zero-copy path, which N ranks on one socket share.
    ``threads`` 0 = min(16, the rank's CPUs)."""
    import ctypes as C
    from ccfd_demo_summit_amd.engine import PinnedArray
    L = lib_()
    ncpu = len(os.sched_getaffinity(0))
    threads = max(1, min(threads or 16, ncpu, 256))
    buf = PinnedArray((mb << 20) // 4, "float32")
    try:
        buf.array[:] = 1.0                     # first touch on this node
        gbps = float(L.ccfd_host_read_bw(C.c_void_p(buf.ptr), mb << 20, threads, seconds))
    finally:
        buf.free()
    return (gbps if gbps > 0 else None), threads


def node_leads(places):
    """{(host, numa_node): lowest rank placed there} for a list of (rank, host, node)."""
    leads = {}
    for rank, host, node in places:
        key = (host, node)
        leads[key] = min(rank, leads.get(key, rank))
    return leads


def host_dram_ceiling(per_rank, row_bytes: int):
    """Aggregate the host-DRAM probes into the zero-copy row ceiling of the whole job.

    Per (host, NUMA node) two lower bounds on what that node's DRAM can feed:
    - ``concurrent_sum``: the SUM of its ranks' ``host_numa_read_GBps``, probed concurrently in
      one barrier-aligned window (each rank saw only its share, so the max would understate
      the node -- the round-3 dp8 rehearsal read 12.9-78.1 GB/s a rank vs 411 alone);
    - ``lead_probe``: the node's lowest rank probing alone with the node's threads
      (``host_node_probe_GBps``) while its other ranks wait at a barrier.
    The node's figure is the larger of the two; the ceiling sums the nodes.  Returns
    (per-node dict, ceiling tx/s or None)."""
    nodes = {}
    for r in per_rank:
        key = f"{r.get('host', '?')}:{r.get('numa_node')}"
        n = nodes.setdefault(key, {"ranks": [], "concurrent_sum": 0.0, "lead_probe": None})
        n["ranks"].append(r.get("rank"))
        if r.get("host_numa_read_GBps") is not None:
            n["concurrent_sum"] += float(r["host_numa_read_GBps"])
        if r.get("host_node_probe_GBps") is not None:
            n["lead_probe"] = max(float(r["host_node_probe_GBps"]), n["lead_probe"] or 0.0)
    for n in nodes.values():
        n["concurrent_sum"] = round(n["concurrent_sum"], 2)
        n["GBps"] = round(max(n["concurrent_sum"], n["lead_probe"] or 0.0), 2)
    tot = sum(n["GBps"] for n in nodes.values())
    return (nodes or None), (round(tot * 1e9 / row_bytes, 1) if tot > 0 else None)


def _encode_cost(args, dm, rows: int):
    """Untimed: host ns per row of the ingest encoder that produced the partition logs' rows
    (W64 bf16 packing, or the G20 / G32 binning against the ensemble's split table -- the
    `x > thr` half of tree evaluation), single thread, SIMD encoder and (binned formats) the
    scalar binary-search encoder it replaced.  The timed region scores pre-encoded rows; this
    puts the encoding cost on the books."""
    import ctypes as C
    from ccfd_demo_summit_amd.data import generate
    from ccfd_demo_summit_amd.ops._lib import lib as _l
    L = _l()
    X, _ = generate(rows, seed=args.seed + 31337)

    def best(fn, a, reps=3):
        t = float("inf")
        for _ in range(reps):
            t0 = time.perf_counter()
            fn(*a)
            t = min(t, time.perf_counter() - t0)
        return t / rows * 1e9
    if args.wire == "f32":
        return {"row_format": "f32", "host_encode_ns_per_row": 0.0}
    if args.wire == "w64":
        out = np.empty((rows, 64), np.uint8)
        ns = best(L.ccfd_encode_w64, (X.ctypes.data, rows, 30, C.c_void_p(out.ctypes.data)))
        return {"row_format": "w64", "host_encode_ns_per_row": round(ns, 2)}
    spec = dm.bins
    flat, offs = spec.flat, spec.offsets
    rb = 20 if args.wire == "g20" else 32
    out = np.empty((rows, rb), np.uint8)
    a = (X.ctypes.data, rows, 30, flat.ctypes.data, offs.ctypes.data, int(spec.stamp), C.c_void_p(out.ctypes.data), None)
    fn, ref = ((L.ccfd_encode_g20, L.ccfd_encode_g20_ref) if args.wire == "g20"
               else (L.ccfd_encode_g32, L.ccfd_encode_g32_ref))
    ns = best(fn, a)
    ns_ref = best(ref, a, reps=1)
    ne = np.diff(offs)
    isa = {2: "avx512", 1: "avx2", 0: "scalar"}.get(int(L.ccfd_encode_isa(int(args.wire == "g20"))), "?")
    return {"row_format": args.wire, "host_encode_ns_per_row": round(ns, 2), "host_encode_isa": isa,
            "host_encode_ns_per_row_scalar_ref": round(ns_ref, 2),
            "max_thresholds_per_feature": int(ne.max()), "mean_thresholds_per_feature": round(float(ne.mean()), 2)}


def _kernel_name(model: str, exec_mode: str, wire: str) -> str:
    """The device kernel a (model, exec mode, row format) engine dispatches (csrc/kernels/)."""
    if exec_mode == "persistent":
        return {"mlp": "persist_kernel<MLP> (score_persist.hip)", "lr": "persist_kernel<LR> (score_persist.hip)",
                "gbdt": "persist_gbdt_g32_kernel (score_gbdt_g32_persist.hip)"}[model]
    if model == "gbdt":
        return "score_gbdt_g32_kernel" if wire in ("g32", "g20") else "score_gbdt_kernel"
    return {"mlp": "score_mlp_wire multi-batch kernel" if wire == "w64" else "score_mlp multi-batch kernel",
            "lr": "score_lr_wire_multi_kernel" if wire == "w64" else "score_lr_multi_kernel"}[model]


def _precision(model, dm, args, dev, exec_mode):
    """Device vs the fp32 oracle on ``--precision-rows`` rows, scored by the SAME engine
    configuration as the timed region (exec mode, row format, input / output modes, depth,
    streams, micro-batch, persistent grid): the rows are replayed from a pinned partition log
    and every row's proba_1 / route comes back through the engine's scored-record ring (the
    kernel's own per-row outputs), matched to the oracle by transaction id."""
    from ccfd_demo_summit_amd.data import generate
    from ccfd_demo_summit_amd.engine import PartitionLog, StreamEngine
    n = max(args.batch, (int(args.precision_rows) // args.batch) * args.batch)
    X, _ = generate(n, seed=args.seed + 4242)
    log = PartitionLog(n, wire=args.wire == "w64", bins=dm.bins)
    if log.row_format != "f32":
        log.write_rows(0, X)
    else:
        log.feats.array[:] = X
    log.ids.array[:] = np.arange(n, dtype=np.uint64)
    eng = StreamEngine(dm, batch=args.batch, depth=args.depth, streams=args.streams,
                       input_mode=args.input_mode, output_mode=args.output_mode, threshold=args.threshold,
                       device=dev.index, exec_mode=exec_mode, persist_grid=args.persist_grid,
                       coalesce=args.coalesce)
    try:
        eng.enable_scored(n)
        eng.add_log(0, log)
        eng.pump(n // args.batch, drain=True)
        rec = eng.drain_scored()
        dropped = eng.scored_dropped()
    finally:
        eng.close()
        log.free()
    ids = rec["tx_id"].astype(np.int64)
    if len(rec) != n or dropped or not np.array_equal(np.sort(ids), np.arange(n)):
        raise RuntimeError(f"precision run: {len(rec)} scored records for {n} rows (dropped {dropped})")
    pd = np.empty(n, np.float64)
    rd = np.empty(n, bool)
    pd[ids] = rec["proba"]
    rd[ids] = rec["route"] != 0
    p32 = model.predict_proba(X).astype(np.float64)
    r32 = (p32 >= args.threshold)
    dp = np.abs(pd - p32)
    flips = (rd != r32)
    outside = np.abs(p32 - args.threshold) > 1e-2
    return {"rows": n, "oracle": "fp32 numpy predict_proba on the unquantised f32 rows",
            "kernel": _kernel_name(args.model, exec_mode, args.wire), "exec_mode": exec_mode,
            "row_format": args.wire, "input_mode": args.input_mode, "output_mode": args.output_mode,
            "depth": args.depth, "micro_batch": args.batch,
            "path": "StreamEngine.pump over a pinned partition log -> scored-record ring (same engine "
                    "configuration as the timed region)",
            "max_abs_dp": float(dp.max()), "mean_abs_dp": float(dp.mean()),
            "route_flips": int(flips.sum()), "route_flip_rate": float(flips.mean()),
            "route_flips_outside_1e-2_band": int((flips & outside).sum()),
            "fraud_routed_fp32": int(r32.sum()), "fraud_routed_device": int(rd.sum())}


def _f32_wire_rate(args, model, dev, exec_mode, seconds: float = 0.5):
    """Secondary run: same model on 30 x f32 (120 B) rows, same engine knobs; tx/s only."""
    from ccfd_demo_summit_amd.data import generate
    from ccfd_demo_summit_amd.engine import PartitionLog, StreamEngine
    from ccfd_demo_summit_amd.ops.kernels import DeviceModel
    dm32 = DeviceModel(model, dev)
    if args.model == "gbdt":
        exec_mode = "launch"                # the persistent GBDT kernel reads binned rows only
    rows = 1 << 20
    log = PartitionLog(rows)
    generate(rows, seed=args.seed + 77, out=log.feats.array)
    log.ids.array[:] = np.arange(rows, dtype=np.uint64)
    eng = StreamEngine(dm32, batch=args.batch, depth=args.depth, streams=args.streams,
                       input_mode=args.input_mode, output_mode=args.output_mode, threshold=args.threshold,
                       device=dev.index, exec_mode=exec_mode, persist_grid=args.persist_grid,
                       coalesce=args.coalesce)
    eng.add_log(0, log)
    eng.pump(256, drain=True)
    t0 = time.perf_counter()
    n = 0
    while time.perf_counter() - t0 < seconds:
        n += eng.pump(512, drain=False).rows
    n += eng.pump(0, drain=True).rows
    dt = time.perf_counter() - t0
    eng.close()
    log.free()
    return n / dt


def main(argv=None):
    args = parse_args(argv)
    from ccfd_demo_summit_amd.utils import benchenv
    refused = benchenv.refusal(allow=args.diagnostic)
    if refused:
        _fail(refused)
    env_block = benchenv.describe()
    diagnostic = bool(env_block["diagnostic"])
    from ccfd_demo_summit_amd.parallel.dp import resolve_row_format
    try:
        args.wire = resolve_row_format(args.model, args.wire)   # auto: w64 for mlp/lr, g20 for gbdt
    except ValueError as e:
        _fail(str(e))
    if args.batch is None:
        args.batch = 65536 if args.model == "gbdt" else 4096
    if args.depth is None:
        # gbdt: 3 micro-batches saturate PCIe for BASELINE's 100 x 6; ensembles past 1200 tree
        # levels a row are VALU-bound and need 6 in flight (profiles/r2/g32_large_ensembles/)
        # G20 rows (1.6x the rows per byte of G32): 4 in flight (2.51e9 vs 2.31e9 tx/s at 3,
        # profiles/r2/g20/sweep.txt)
        args.depth = (6 if args.gbdt_trees * args.gbdt_depth > 1200 else 4 if args.wire == "g20" else 3) \
            if args.model == "gbdt" else 12
    import torch
    from ccfd_demo_summit_amd.data import FRAUD_RATE, generate
    from ccfd_demo_summit_amd.engine import FlaggedDrainer, PartitionLog, StreamEngine
    from ccfd_demo_summit_amd.models import build_model
    from ccfd_demo_summit_amd.ops._lib import lib
    from ccfd_demo_summit_amd.parallel import (CounterReducer, EpochPipeline, all_max, assign_partitions,
                                               barrier, broadcast_model, hist_quantile, init_distributed)

    if not torch.cuda.is_available():
        raise SystemExit("bench.py needs a GPU (MI355X)")
    ctx = init_distributed(timeout_s=args.pg_timeout_s)
    dev = ctx.device
    W = ctx.world
    idents, problems = _verify_topology(args, ctx, _device_ident(ctx, dev))
    # ---- watchdog: a rank with no completed step for --watchdog-s prints its state and exits
    # non-zero (a wedged RCCL collective or doorbell would otherwise sit until the PG timeout)
    from ccfd_demo_summit_amd.utils.faults import FaultPlan
    from ccfd_demo_summit_amd.utils.watchdog import Watchdog
    wd_state = {"phase": "setup", "last_collective": None}
    faults = FaultPlan.from_env(ctx.rank)

    def _wd_report():
        st = dict(wd_state)
        e = wd_state.get("engine")
        st.pop("engine", None)
        ep = wd_state.get("epochs")
        st.pop("epochs", None)
        if e is not None:
            st["engine"] = e.progress()
        if ep is not None:
            st["x2_ticks"] = ep.ticks
            st["x2_reducer_busy"] = ep.reducer.busy()
            st["x2_reductions"] = ep.reducer.epochs
        return st
    watchdog = Watchdog(args.watchdog_s, _wd_report, rank=ctx.rank, name="bench").start()
    from ccfd_demo_summit_amd.utils.numa import bind_to_gpu
    numa_node = bind_to_gpu(dev.index)     # pinned logs + host threads on the GPU's socket

    # ---- model: rank 0 builds (random init of the named architecture; normaliser fitted and
    # output bias calibrated on a synthetic sample so ~0.17 % of traffic routes to the fraud
    # process, like the dataset prior), X1 broadcast over RCCL to every rank.
    model = None
    if ctx.rank == 0:
        Xcal, _ = generate(200_000, seed=args.seed + 999)
        model = build_model(args.model, seed=args.seed, X_ref=Xcal, calibrate_rate=FRAUD_RATE,
                            threshold=args.threshold, gbdt_trees=args.gbdt_trees, gbdt_depth=args.gbdt_depth)
    dm = broadcast_model(ctx, model, args.model, args.wire)     # X1 (+ the G32 bin table)
    args.wire = dm.row_format          # G32 falls back to f32 rows for unbinnable ensembles
    bins = dm.bins
    exec_mode = args.exec_mode
    if exec_mode == "auto":
        # measured on MI355X (profiles/r1/persist_sweep.txt): the persistent kernel with a
        # parallel doorbell and 512-row work items reaches 0.82e9 tx/s at p50 147 us, above
        # coalesced launches (0.75e9 at 166 us); GBDT on G32 rows: 1.68e9 persistent vs 1.07e9
        # with launches (profiles/r2/gbdt_g32_*_sweep.jsonl); DMA paths use launches
        zc = args.input_mode == "zerocopy" and args.output_mode == "zerocopy"
        exec_mode = "persistent" if zc and (args.model in ("mlp", "lr") or args.wire in ("g32", "g20")) else "launch"

    # ---- per-rank H2D ceiling probe, all ranks at once (attributes any scaling loss to the
    # host side: DRAM / PCIe root contention shows up as a lower per-rank GB/s at N > 1)
    h2d_gbps = None
    if args.probe_ms > 0 and args.input_mode == "zerocopy":
        wd_state["last_collective"] = "barrier:h2d_probe"
        barrier(ctx)
        h2d_gbps = _h2d_probe(lib, args.probe_ms)
    # ---- CPU-side DRAM read probe of each rank's NUMA node, all ranks at once: what the
    # sockets can feed N zero-copy ranks (8 x ~55 GB/s over two sockets)
    # phase 1: every rank at once (each sees its share of its node); phase 2: the lowest rank
    # of each (host, node) alone with the node's threads while the node's other ranks wait
    host_bw = host_threads = node_bw_lead = node_threads = None
    if args.host_probe_s > 0:
        wd_state["last_collective"] = "barrier:host_probe"
        barrier(ctx)
        host_bw, host_threads = _host_read_probe(lib, args.host_probe_s)
        places = [(ctx.rank, idents[ctx.rank if ctx.initialized else 0]["host"], numa_node)]
        if ctx.initialized:
            import torch.distributed as dist
            places = [None] * W
            dist.all_gather_object(places, (ctx.rank, idents[ctx.rank]["host"], numa_node))
        lead = node_leads(places)[(places[ctx.rank if ctx.initialized else 0][1], numa_node)] == ctx.rank
        wd_state["last_collective"] = "barrier:host_node_probe"
        barrier(ctx)
        if lead:
            node_bw_lead, node_threads = _host_read_probe(lib, args.host_probe_s, threads=32)
        barrier(ctx)
    watchdog.beat("probes")

    # ---- this rank's partitions of topic odh-demo (p % W == rank), pre-filled logs
    n_parts = args.partitions_per_rank * W
    my_parts = assign_partitions(n_parts, ctx.rank, W)
    rows_per_part = max(args.batch * 4, args.log_rows // len(my_parts))
    logs = []
    eng = StreamEngine(dm, batch=args.batch, depth=args.depth, streams=args.streams,
                       input_mode=args.input_mode, output_mode=args.output_mode,
                       threshold=args.threshold, device=dev.index, exec_mode=exec_mode,
                       persist_grid=args.persist_grid, coalesce=args.coalesce,
                       flag_capacity=args.flag_capacity)
    for p in my_parts:
        log = PartitionLog(rows_per_part, wire=args.wire == "w64", bins=bins)
        if log.row_format != "f32":
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
    bps = [args.batches_per_step]
    x2_every = [max(1, args.x2_every or 8)]

    rows_local = [0]

    wd_state.update(engine=eng, epochs=epochs, phase="warmup")
    watchdog.on_fire = lambda: eng.emergency_stop(5000)     # never exit with a resident kernel
    if faults is not None:
        faults.before_exit = lambda: eng.emergency_stop(5000)
    import signal

    def _term(signum, _frame):                 # an outer SIGTERM: the kernel leaves first
        eng.emergency_stop(5000)
        os._exit(128 + signum)
    signal.signal(signal.SIGTERM, _term)

    handoff_mu = threading.Lock()

    def handoff(records):
        # router hand-off of fraud-routed transactions (transaction.outgoing{type=fraud});
        # called by the collector thread and, on a full ring, by the pump's thread
        nonlocal flagged_total
        with handoff_mu:
            flagged_total += len(records)

    # the router's collector: a thread drains the flagged ring while this thread keeps the
    # micro-batches coming (as the streaming service's native serving thread + collector do);
    # draining inline between steps idled the GPU for every drain (profiles/r6/pass_h/)
    drainer = FlaggedDrainer(eng, handoff).start()

    def step(drain: bool):
        if faults is not None:
            faults.step()                  # CCFD_FAULTS (utils/faults.py): delay / stall / crash a rank
        # a full flagged ring stops the pump (nothing retired, nothing lost), the hand-off drains
        # it and the pump resumes: every fraud-routed row is handed off exactly once
        rows_local[0] += eng.pump(bps[0], drain=drain, on_flagged=handoff).rows
        nstep[0] += 1
        if nstep[0] % x2_every[0]:
            return
        # X2/X3: flip the counter epoch; the previously closed epoch (all of whose batches
        # have completed by now) is all-reduced over RCCL on the side stream
        tx = time.perf_counter()
        wd_state["last_collective"] = f"x2_all_reduce#{epochs.ticks}"
        epochs.tick(progress=lambda: eng.run(0, 0))   # (retire finished batches if it must wait)
        x2_s[0] += time.perf_counter() - tx
        watchdog.beat(f"step {nstep[0]}")

    for _ in range(args.warmup):
        step(drain=False)
        watchdog.beat("warmup step")
    wd_state["phase"] = "calibration"
    # ---- calibration (untimed): size a step so the K timed steps are a sustained run of at
    # least --min-timed-s; every rank takes the max, so all ranks run the same work
    tc = time.perf_counter()
    cal_steps = 4
    for _ in range(cal_steps):
        step(drain=False)
        watchdog.beat("calibration step")
    wd_state["last_collective"] = "all_max:calibration"
    per_batch_s = all_max(ctx, (time.perf_counter() - tc) / (cal_steps * bps[0]))
    need = int(np.ceil(args.min_timed_s * 1.05 / max(1, args.steps) / max(per_batch_s, 1e-9)))
    bps[0] = max(args.batches_per_step, need)
    step_s_est = bps[0] * per_batch_s
    x2_every[0] = args.x2_every or max(1, int(round(args.x2_period_ms / 1e3 / max(step_s_est, 1e-9))))
    eng.pump(0, drain=True)
    epochs.finish()
    eng.reset_stats()
    if args.trace and ctx.rank == 0:
        eng.enable_trace(65536)
    c0 = reducer.snapshot()[0]
    rows0, fraud0 = int(c0[0]), int(c0[1])
    drainer.stop()               # warmup hand-offs are not part of the timed run
    flagged_total = 0
    drainer.records = drainer.drains = 0
    full0 = eng.pump(0, drain=False).flag_full_events
    x2_s[0] = 0.0
    nstep[0] = 0
    rows_local[0] = 0
    wd_state["last_collective"] = "barrier:timed_start"
    barrier(ctx)
    torch.cuda.synchronize(dev)
    wd_state["phase"] = "timed"

    t0 = time.perf_counter()
    drainer.start()
    for k in range(args.steps):
        step(drain=(k == args.steps - 1))
        watchdog.beat(f"timed step {k}")
    drainer.stop()               # every fraud record of the timed batches handed off in the region
    wd_state["last_collective"] = "x2_finish"
    epochs.finish()
    torch.cuda.synchronize(dev)
    t_local = time.perf_counter() - t0
    wd_state["last_collective"] = "barrier:timed_end"
    barrier(ctx)
    wd_state["phase"] = "report"
    watchdog.beat("timed region done")
    t1 = time.perf_counter()
    elapsed = all_max(ctx, t1 - t0)

    # latency: per-rank histogram of the timed batches, merged over ranks (X3)
    st_final = eng.pump(0, drain=True, on_flagged=handoff)
    rows_local[0] += st_final.rows
    handoff(eng.drain_flagged())
    handoff_stalls = st_final.flag_full_events - full0
    if args.trace and ctx.rank == 0:
        from ccfd_demo_summit_amd.utils.tracing import dump_batch_trace
        dump_batch_trace(eng.read_trace(), args.trace, name=f"engine rank 0 ({args.model})")
    lat_local = st_final.lat_hist.astype(np.int64)
    lat_t = torch.from_numpy(lat_local).to(dev)
    if ctx.initialized:
        import torch.distributed as dist
        dist.all_reduce(lat_t)
    lat = lat_t.cpu().numpy()
    counters, _ = reducer.snapshot()
    total_rows = int(counters[0] - rows0)
    expected = args.steps * bps[0] * args.batch * W
    p50_us = hist_quantile(lat, 0.50) / 1e3
    p99_us = hist_quantile(lat, 0.99) / 1e3
    nb_local = args.steps * bps[0]
    rank_info = {
        "rank": ctx.rank, "pci": idents[ctx.rank]["pci"] if ctx.initialized else idents[0]["pci"],
        "host": (idents[ctx.rank] if ctx.initialized else idents[0])["host"],
        "numa_node": numa_node,
        "rows": int(rows_local[0]),
        "tx_s": round(rows_local[0] / t_local, 1) if t_local > 0 else None,
        "local_timed_s": round(t_local, 4),
        "p50_latency_us": round(hist_quantile(lat_local, 0.5) / 1e3, 2),
        "device_exec_us_p50": round(hist_quantile(st_final.dev_hist.astype(np.int64), 0.5) / 1e3, 2)
        if st_final.dev_batches else None,
        "host_wait_us_per_batch": round(st_final.host_wait_s * 1e6 / nb_local, 3),
        "h2d_zerocopy_GBps": None if h2d_gbps is None else round(h2d_gbps, 2),
        "host_numa_read_GBps": None if host_bw is None else round(host_bw, 2),
        "host_probe_threads": host_threads,
        "host_node_probe_GBps": None if node_bw_lead is None else round(node_bw_lead, 2),
        "host_node_probe_threads": node_threads,
        "flagged_handed_off": int(flagged_total),
        "handoff_stalls": int(handoff_stalls),
        "handoff_drains": int(drainer.drains),
    }
    per_rank = [rank_info]
    if ctx.initialized:
        import torch.distributed as dist
        per_rank = [None] * W
        dist.all_gather_object(per_rank, rank_info)

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
    eng.close()
    for log in logs:
        log.free()

    # precision evidence + f32-row throughput (rank 0, after the timed region)
    precision = f32_rate = encode = None
    if ctx.rank == 0:
        if args.precision_rows > 0:
            precision = _precision(model, dm, args, dev, exec_mode)
        if args.encode_probe_rows > 0:
            encode = _encode_cost(args, dm, args.encode_probe_rows)
        if args.wire in ("w64", "g32", "g20") and not args.no_f32_probe:
            f32_rate = _f32_wire_rate(args, model, dev, exec_mode)

    flagged_all = sum(r["flagged_handed_off"] for r in per_rank)
    value = total_rows / elapsed
    base = baseline_value()
    row_b = {"w64": 64, "g32": 32, "g20": 20, "f32": 120}[args.wire]
    # host ceiling of the zero-copy row stream: a scaling loss at N > 1 that this predicts is
    # the host side, not the GPUs or RCCL
    node_bw, host_ceiling = host_dram_ceiling(per_rank, row_b)
    if encode is not None and encode.get("host_encode_ns_per_row"):
        # host threads needed to encode the stream at the measured rate (the ingest side of a
        # deployment does this in the Kafka consumer threads, csrc/engine/kafka_consumer.cpp)
        encode["encode_threads_needed_at_value"] = round(value * encode["host_encode_ns_per_row"] * 1e-9, 2)
    rehearsal = bool(problems)
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
        # context only: config 1 is OUR CPU batch=1 LR REST measurement, not a
        # published reference number and not the same model
        "vs_baseline": (round(value / base, 1) if base else None),
        "vs_baseline_note": "ratio to config 1 (CPU LR batch=1 Seldon REST, measured by us); "
                            "the reference publishes no numbers",
        "dtype": "bf16" if args.model == "mlp" else "fp32",
        "data": ("synthetic creditcard-shaped transactions (30 features; log rows "
                 + {"w64": "W64: bf16 V1..V28 + f32 Time/Amount, 64 B",
                    "g32": "G32: u8 bin of each feature against the ensemble's split thresholds "
                           "(exact for oblivious trees) + amount bucket + table stamp, 32 B",
                    "g20": "G20: 5-bit bin of each feature against the ensemble's split thresholds "
                           "(exact for oblivious trees, <= 31 a feature) + amount bucket + table stamp, 20 B",
                    "f32": "30 x f32, 120 B"}[args.wire]
                 + ") replayed from pinned partition logs; random-init weights, normaliser fitted + "
                 "output bias calibrated to the 0.172% fraud prior on a synthetic sample"),
        "config": {"model": {"mlp": "mlp_30_128_64_1", "lr": "logreg_30",
                             "gbdt": f"oblivious_gbdt_{args.gbdt_trees}x{args.gbdt_depth}"}[args.model],
                   "global_batch": args.batch * W, "seq_len": 1, "micro_batch": args.batch,
                   "parallelism": f"dp{W}" + ("-rehearsal" if rehearsal else "") + ("-diagnostic" if diagnostic else ""),
                   "input_mode": args.input_mode,
                   "output_mode": args.output_mode, "exec_mode": exec_mode, "depth": args.depth,
                   "wire": args.wire, "coalesce": args.coalesce,
                   "streams": args.streams,
                   "batches_per_step": bps[0], "x2_every_steps": x2_every[0],
                   "numa_node_rank0": numa_node},
        "timed_region_s": round(elapsed, 4),
        "backend": ctx.backend,
        "world_size": W,
        "rehearsal": rehearsal,
        "topology_problems": problems,
        # every CCFD_* / HIP_* / HSA_* / ... variable this rank saw; a diagnostic one makes the
        # run refuse unless --diagnostic, which labels the line (utils/benchenv.py)
        "diagnostic": diagnostic,
        "env": env_block,
        "p50_latency_us": round(p50_us, 2),
        "p99_latency_us": round(p99_us, 2),
        "p50_latency_us_unloaded": None if p50_unloaded is None else round(p50_unloaded, 2),
        # engine host-thread time per timed micro-batch (cumulative since reset_stats)
        "host_us_per_batch": {k: round(v * 1e6 / nb_local, 3) for k, v in
                              (("submit", st_final.host_submit_s), ("wait", st_final.host_wait_s),
                               ("complete", st_final.host_complete_s))},
        # host time per step spent in the X2 tick (epoch flip + side-stream all-reduce issue)
        "host_us_per_step_x2": round(x2_s[0] * 1e6 / args.steps, 2),
        "step_us_per_batch": round(elapsed * 1e6 / nb_local, 3),
        # K7: per-micro-batch execution window on the GPU's own clock (rank 0)
        "device_exec_us_mean": round(st_final.dev_exec_mean_us, 2),
        "device_exec_us_p50": rank_info["device_exec_us_p50"],
        "device_exec_us_p99": (round(hist_quantile(st_final.dev_hist.astype(np.int64), 0.99) / 1e3, 2)
                               if st_final.dev_batches else None),
        "rows_scored": total_rows,
        "rows_expected": expected,
        "fraud_routed": int(counters[1]) - fraud0,
        "wire_stale_rows": int(counters[4]),      # G32 rows refused for a foreign bin-table stamp
        "flagged_handed_off_rank0": flagged_total,
        # sum over ranks; must equal fraud_routed (the bench refuses to print the line otherwise)
        "flagged_handed_off": flagged_all,
        # pumps stopped on a full flagged ring during the timed region (stall, not loss)
        "handoff_stalls": sum(r["handoff_stalls"] for r in per_rank),
        # the hand-off runs on a collector thread beside the pump (FlaggedDrainer), inside the
        # timed region; every record counted before the clock stops
        "handoff": "collector thread",
        "per_rank": per_rank,
        "h2d_zerocopy_ceiling_tx_s_rank0": (None if h2d_gbps is None else
                                            round(h2d_gbps * 1e9 / row_b, 1)),
        # CPU streaming-read GB/s per (host, NUMA node): concurrent per-rank sum and the node
        # lead's all-thread probe (host_dram_ceiling), and the zero-copy row ceiling they imply
        "host_numa_read_GBps": node_bw,
        "host_dram_ceiling_tx_s": host_ceiling,
        "host_encode": encode,
        "f32_wire_tx_s": None if f32_rate is None else round(f32_rate, 1),
        "precision_vs_fp32": precision,
        "timed_kernel": _kernel_name(args.model, exec_mode, args.wire),
    }
    if total_rows != expected and ctx.rank == 0:
        print(f"[bench] WARNING: counted {total_rows} rows, expected {expected}", file=sys.stderr)
    # lossless hand-off: every fraud-routed row of the timed region reached the router hand-off
    # exactly once; a line where it did not would count hand-off work that was skipped
    refused = handoff_refusal(flagged_all, out["fraud_routed"])
    lossless = refused is None
    if not lossless and ctx.rank == 0:
        print(f"[bench] FATAL: {refused}", file=sys.stderr, flush=True)
    if ctx.rank == 0 and lossless:
        line = json.dumps(out)
        print(line, flush=True)
        if args.out:
            Path(args.out).write_text(line + "\n")
    watchdog.stop()
    if ctx.initialized:
        import torch.distributed as dist
        barrier(ctx)
        dist.destroy_process_group()
    if total_rows != expected or int(counters[4]) != 0:
        raise SystemExit(4)
    if not lossless:
        raise SystemExit(5)


def handoff_refusal(flagged_handed_off: int, fraud_routed: int):
    """None when every fraud-routed row of the timed region was handed off exactly once, else
    why the run must not be reported: a line with fewer hand-offs than routed rows skipped
    hand-off work inside the timed region."""
    if flagged_handed_off == fraud_routed:
        return None
    return (f"handed off {flagged_handed_off} fraud records, the kernels routed {fraud_routed}: "
            "refusing to report this run")


def entry(argv=None) -> int:
    """``python bench.py --gpus N``: at N > 1 with no WORLD_SIZE in the env, this process is
    only the parent -- it runs ``torch.distributed.run --nproc-per-node N bench.py <argv>`` as
    a child (never exec, never touching the GPU itself), forwards rank 0's JSON line and
    returns the worst rank's exit code (launch/local_ranks.py).  Otherwise it is a rank."""
    argv = list(sys.argv[1:] if argv is None else argv)
    from ccfd_demo_summit_amd.launch import local_ranks
    args = parse_args(argv)
    from ccfd_demo_summit_amd.utils import benchenv
    refused = benchenv.refusal(allow=args.diagnostic)
    if refused:
        print(f"[bench] FATAL: {refused}", file=sys.stderr, flush=True)
        return 3
    if local_ranks.needs_spawn(args.gpus):
        env = dict(local_ranks.REHEARSAL_ENV) if args.rehearsal else {}
        return local_ranks.run_ranks(str(Path(__file__).resolve()), argv, args.gpus, extra_env=env)
    code = 0
    try:
        main(argv)
    except SystemExit as e:
        code = e.code if isinstance(e.code, int) else (0 if e.code is None else 1)
        raise
    except BaseException:
        code = 1
        raise
    finally:
        local_ranks.record_rank_rc(code)
    return 0


if __name__ == "__main__":
    sys.exit(entry())
