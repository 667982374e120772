#!/usr/bin/env python3
"""Zero-copy read bandwidth from pinned host memory on 4 KB pages (hipHostMalloc) vs
transparent huge pages (ccfd_host_alloc_huge: 2 MB-aligned, MADV_HUGEPAGE, hipHostRegister),
for the streaming pattern (one big grid-stride read) and for scattered per-workgroup blocks
(the persistent kernel's small items: 4 / 8 / 32 KB per workgroup at a time).  One JSON line
per (allocation, pattern).

    python bench/experiments/pinned_pages.py [--mb 1024]
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mb", type=int, default=1024)
    ap.add_argument("--iters", type=int, default=8)
    a = ap.parse_args()
    import torch
    from ccfd_demo_summit_amd.ops._lib import lib
    L = lib()
    L.ccfd_host_alloc_huge.restype = C.c_void_p
    L.ccfd_host_alloc_huge.argtypes = [C.c_size_t]
    L.ccfd_bw_probe_blocks.restype = C.c_double
    L.ccfd_bw_probe_blocks.argtypes = [C.c_void_p, C.c_size_t, C.c_size_t, C.c_int, C.c_int, C.c_void_p]
    L.ccfd_bw_probe.restype = C.c_double
    L.ccfd_bw_probe.argtypes = [C.c_void_p, C.c_size_t, C.c_int, C.c_int, C.c_void_p]
    L.ccfd_host_alloc.restype = C.c_void_p
    L.ccfd_host_alloc.argtypes = [C.c_size_t]
    nbytes = a.mb << 20
    scratch = torch.empty(1 << 16, dtype=torch.uint8, device="cuda")
    thp = Path("/sys/kernel/mm/transparent_hugepage/enabled")
    thp_mode = thp.read_text().strip() if thp.exists() else "n/a"
    allocs = {"hipHostMalloc_4k": L.ccfd_host_alloc(nbytes), "thp_registered": L.ccfd_host_alloc_huge(nbytes)}
    for name, ptr in allocs.items():
        if not ptr:
            print(json.dumps({"alloc": name, "error": "allocation failed"}), flush=True)
            continue
        C.memset(ptr, 1, nbytes)
        r = {"alloc": name, "thp": thp_mode, "mb": a.mb,
             "stream_GBps": round(L.ccfd_bw_probe(C.c_void_p(ptr), nbytes, 1, a.iters, C.c_void_p(scratch.data_ptr())), 2)}
        for blk_kb, grid in ((4, 256), (8, 128), (8, 256), (32, 64), (32, 256)):
            r[f"blocks_{blk_kb}k_grid{grid}_GBps"] = round(
                L.ccfd_bw_probe_blocks(C.c_void_p(ptr), nbytes, blk_kb << 10, grid, a.iters,
                                       C.c_void_p(scratch.data_ptr())), 2)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
