"""Measure the streaming roofline on one GPU: pinned-host -> GPU bandwidth by SDMA copy and
by zero-copy kernel loads, and HBM read bandwidth; print the implied tx/s ceilings for
120-byte (30 x f32) transactions.

    python bench/roofline.py [--mb 256]
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mb", type=int, default=256)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--chunked", action="store_true", help="also probe micro-batch-sized kernels")
    args = ap.parse_args()
    import torch
    from ccfd_demo_summit_amd.engine import PinnedArray
    from ccfd_demo_summit_amd.ops._lib import lib
    L = lib()
    L.ccfd_bw_probe.argtypes = [C.c_void_p, C.c_size_t, C.c_int, C.c_int, C.c_void_p]
    L.ccfd_bw_probe.restype = C.c_double
    nbytes = args.mb << 20
    host = PinnedArray(nbytes // 4, "float32")
    host.array[:] = 1.0
    dev = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    dsrc = torch.ones(nbytes // 4, dtype=torch.float32, device="cuda")
    out = {}
    out["h2d_sdma_GBps"] = L.ccfd_bw_probe(C.c_void_p(host.ptr), nbytes, 0, args.iters, C.c_void_p(dev.data_ptr()))
    out["h2d_zerocopy_kernel_GBps"] = L.ccfd_bw_probe(C.c_void_p(host.ptr), nbytes, 1, args.iters,
                                                      C.c_void_p(dev.data_ptr()))
    out["hbm_read_GBps"] = L.ccfd_bw_probe(C.c_void_p(dsrc.data_ptr()), nbytes, 2, args.iters,
                                           C.c_void_p(dev.data_ptr()))
    for k in list(out):
        out[k.replace("_GBps", "_tx_ceiling_M_per_s")] = round(out[k] * 1e9 / 120 / 1e6, 1)
        out[k] = round(out[k], 2)
    if args.chunked:
        # micro-batch granularity: chunk = rows x 120 B, grid/block like the scoring kernels
        L.ccfd_bw_probe_chunked.argtypes = [C.c_void_p, C.c_size_t, C.c_size_t, C.c_int, C.c_int, C.c_int,
                                            C.c_int, C.c_void_p]
        L.ccfd_bw_probe_chunked.restype = C.c_double
        rows_list = [4096, 16384, 65536]
        out["chunked"] = []
        for rows in rows_list:
            chunk = rows * 120
            for grid, block in ((rows // 64, 256), (rows // 16, 64), (min(2048, rows // 16), 256)):
                for ns in (1, 4, 8):
                    gbps = L.ccfd_bw_probe_chunked(C.c_void_p(host.ptr), nbytes, chunk, grid, block, ns, 3,
                                                   C.c_void_p(dev.data_ptr()))
                    out["chunked"].append({"rows": rows, "grid": grid, "block": block, "streams": ns,
                                           "GBps": round(gbps, 2), "tx_M_per_s": round(gbps * 1e9 / 120 / 1e6, 1)})
    print(json.dumps(out))
    host.free()


if __name__ == "__main__":
    main()
