#!/usr/bin/env python3
"""Speed-of-light check of the fused scoring kernels on HBM-resident rows.

The streaming headline (bench.py) is bound by PCIe bytes per transaction
(profiles/r1/roofline.json), so it cannot tell whether the kernels themselves are fast.
This bench removes PCIe: rows live in HBM, one launch scores ``B`` rows, and the time is
compared with the two ceilings of the kernel on MI355X:

* HBM: bytes read + written per row / measured HBM read bandwidth (bench/roofline.py);
* MFMA (MLP only): 26 ``mfma_f32_16x16x32_bf16`` per 16 rows = 26.6 KFLOP/row against the
  dense bf16 peak (2.5 PFLOP/s, no sparsity).

    python bench/kernel_sol.py [--out profiles/r1/kernel_sol.json]
    python bench/kernel_sol.py --cases mlp:w64 --sizes 16777216 --flags 48   # ablation
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

HBM_GBPS_MEASURED = 7071.5          # profiles/r1/roofline.json hbm_read_GBps
BF16_DENSE_TFLOPS = 2500.0
MLP_FLOP_PER_ROW = 26 * 16 * 16 * 32 * 2 / 16     # padded MFMA work actually issued (8 + 16 + 2 per 16 rows)


class _HostRows:
    """Quacks like the CUDA row tensor score() expects, but points at pinned host memory
    (the device alias of a PinnedArray): the kernel reads it zero-copy over PCIe."""

    def __init__(self, pinned, n, cols, dtype):
        from ccfd_demo_summit_amd.ops._lib import lib
        import torch
        self._p, self.shape, self.dtype = pinned, (n, cols), dtype
        self._ptr = lib().ccfd_host_device_ptr(pinned.ptr)
        self.is_cuda, self.device = True, torch.device("cuda", 0)

    def dim(self):
        return 2

    def element_size(self):
        import torch
        return torch.empty(0, dtype=self.dtype).element_size()

    def is_contiguous(self):
        return True

    def stride(self, d):
        return (self.shape[1], 1)[d]

    def data_ptr(self):
        return self._ptr


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="4096,65536,1048576,16777216")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--cases", default="mlp:w64,mlp:f32,lr:w64,lr:f32,gbdt:f32")
    ap.add_argument("--flags", type=int, default=0, help="extra CCFD_ARG_* bits (16 = no counter atomics, "
                    "32 = no proba/route stores)")
    ap.add_argument("--tag", default="", help="label copied into every result line")
    ap.add_argument("--host", action="store_true",
                    help="rows in pinned host memory read zero-copy over PCIe (the streaming input path) "
                         "instead of HBM: one launch per size, no engine")
    ap.add_argument("--gbdt-trees", type=int, default=100)
    ap.add_argument("--gbdt-depth", type=int, default=6)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    import torch
    from ccfd_demo_summit_amd.contracts.transaction import encode_wire
    from ccfd_demo_summit_amd.data import generate
    from ccfd_demo_summit_amd.models import build_model
    from ccfd_demo_summit_amd.ops.kernels import DeviceModel, new_counters, score

    dev = torch.device("cuda", 0)
    sizes = [int(s) for s in args.sizes.split(",")]
    cases = [tuple(c.replace("/", ":").split(":")) for c in args.cases.split(",")]   # kind:wire or kind/wire
    nmax = max(sizes)
    X, _ = generate(1 << 20, seed=3)
    reps = (nmax + X.shape[0] - 1) // X.shape[0]
    xf = xw = xg = None
    if any(w == "f32" for _, w in cases):
        xf = torch.from_numpy(X).to(dev).repeat(reps, 1)[:nmax].contiguous()
    if any(w == "w64" for _, w in cases):
        xw = torch.from_numpy(encode_wire(X)).to(dev).repeat(reps, 1)[:nmax].contiguous()
    results = []
    for kind, wire in cases:
        m = build_model(kind, seed=0, X_ref=X[:100_000], calibrate_rate=0.01, gbdt_trees=args.gbdt_trees,
                        gbdt_depth=args.gbdt_depth)
        dm = DeviceModel(m, dev, wire=(wire == "w64"), bins=wire if wire in ("g32", "g20") else None)
        if wire in ("g32", "g20"):
            xg = torch.from_numpy(dm.bins.encode(X)).to(dev).repeat(reps, 1)[:nmax].contiguous()
        x_all = {"w64": xw, "g32": xg, "g20": xg}.get(wire, xf)
        in_bytes = {"w64": 64, "g32": 32, "g20": 20}.get(wire, 120)
        host_rows = None
        if args.host:
            from ccfd_demo_summit_amd.engine import PinnedArray
            host_rows = PinnedArray((nmax, in_bytes // 4), "float32")
            host_rows.array[:] = x_all.view(torch.float32).reshape(nmax, in_bytes // 4).cpu().numpy()
        for n in sizes:
            x = x_all[:n] if host_rows is None else _HostRows(host_rows, n, x_all.shape[1], x_all.dtype)
            proba = torch.empty(n, dtype=torch.float32, device=dev)
            route = torch.empty(n, dtype=torch.uint8, device=dev)
            ctr = new_counters(dev)
            for _ in range(3):
                score(dm, x, proba=proba, route=route, counters=ctr, flags=args.flags)
            torch.cuda.synchronize(dev)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            iters = max(3, min(args.iters * 64, int(args.iters * (1 << 22) / n)))
            e0.record()
            for _ in range(iters):
                score(dm, x, proba=proba, route=route, counters=ctr, flags=args.flags)
            e1.record()
            torch.cuda.synchronize(dev)
            us = e0.elapsed_time(e1) * 1e3 / iters
            rows_s = n / (us * 1e-6)
            gbps = rows_s * (in_bytes + 5) / 1e9
            r = {"tag": args.tag, "flags": args.flags, "model": kind, "wire": wire, "rows": n,
                 "rows_in": "host-zerocopy" if args.host else "hbm",
                 "us_per_launch": round(us, 2), "G_rows_per_s": round(rows_s / 1e9, 3), "GBps": round(gbps, 1),
                 "frac_hbm_roofline": round(gbps / HBM_GBPS_MEASURED, 3)}
            if kind == "mlp":
                tf = rows_s * MLP_FLOP_PER_ROW / 1e12
                r["mfma_TFLOPs"] = round(tf, 1)
                r["frac_bf16_dense_peak"] = round(tf / BF16_DENSE_TFLOPS, 3)
            print(json.dumps(r), flush=True)
            results.append(r)
    if args.out:
        Path(args.out).write_text(json.dumps({"hbm_GBps_ceiling": HBM_GBPS_MEASURED,
                                              "bf16_dense_TFLOPs": BF16_DENSE_TFLOPS,
                                              "results": results}, indent=1) + "\n")


if __name__ == "__main__":
    main()
