"""Zero-copy read rate of pinned host memory against the per-lane load width.

The G20 GBDT rows were fetched with one dword per lane (a 256 B wave request per
instruction) while the W64 MLP tiles use 16 B per lane (1 KB per instruction); this probe
(`ccfd_bw_probe_width`, csrc/kernels/probe.hip) isolates the width's effect on the PCIe
zero-copy rate.  Prints one JSON line per (width, grid).
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--mb", type=int, default=256)
    ap.add_argument("--widths", default="4,8,16")
    ap.add_argument("--grids", default="512,2048")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    import torch
    from ccfd_demo_summit_amd.engine import PinnedArray
    from ccfd_demo_summit_amd.ops._lib import lib
    L = lib()
    L.ccfd_bw_probe_width.argtypes = [C.c_void_p, C.c_size_t, C.c_int, C.c_int, C.c_int, C.c_void_p]
    L.ccfd_bw_probe_width.restype = C.c_double
    nbytes = args.mb << 20
    host = PinnedArray(nbytes // 4, "float32")
    host.array[:] = 1.0
    scratch = torch.empty(1 << 16, dtype=torch.uint8, device="cuda")
    out = open(args.out, "w") if args.out else None
    try:
        for grid in (int(g) for g in args.grids.split(",")):
            for w in (int(x) for x in args.widths.split(",")):
                gbps = L.ccfd_bw_probe_width(C.c_void_p(host.ptr), nbytes, w, grid, args.iters,
                                             C.c_void_p(scratch.data_ptr()))
                rec = {"width_bytes": w, "wave_request_bytes": 64 * w, "grid": grid, "mb": args.mb,
                       "GBps": round(gbps, 2)}
                print(json.dumps(rec), flush=True)
                if out:
                    out.write(json.dumps(rec) + "\n")
    finally:
        host.free()
        if out:
            out.close()


if __name__ == "__main__":
    main()
