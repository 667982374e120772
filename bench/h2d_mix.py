"""Can the pinned-host -> GPU link carry more than one feeder alone?  Sweeps the mixed probe
(csrc/kernels/probe.hip ccfd_bw_probe_mix): a fraction of each pass read zero-copy by a
kernel, the rest copied by 1..N SDMA streams, all concurrently.  One JSON line per point.

    python bench/h2d_mix.py [--mb 512]
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
    ap.add_argument("--mb", type=int, default=512)
    ap.add_argument("--iters", type=int, default=8)
    ap.add_argument("--sdma", default="0,1,2,4")
    ap.add_argument("--zc", default="0,0.25,0.5,0.75,1")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    import torch
    from ccfd_demo_summit_amd.engine import PinnedArray
    from ccfd_demo_summit_amd.ops._lib import lib
    L = lib()
    L.ccfd_bw_probe_mix.argtypes = [C.c_void_p, C.c_size_t, C.c_int, C.c_double, C.c_int, C.c_void_p]
    L.ccfd_bw_probe_mix.restype = C.c_double
    nbytes = args.mb << 20
    host = PinnedArray(nbytes // 4, "float32")
    host.array[:] = 1.0
    dev = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    rows = []
    for n in [int(x) for x in args.sdma.split(",")]:
        for z in [float(x) for x in args.zc.split(",")]:
            if n == 0 and z < 1.0:
                continue
            if z == 1.0 and n > 0:
                continue
            g = L.ccfd_bw_probe_mix(C.c_void_p(host.ptr), nbytes, n, z, args.iters, C.c_void_p(dev.data_ptr()))
            r = {"sdma_streams": n, "zerocopy_fraction": z, "GBps": round(g, 2),
                 "w64_tx_ceiling_M_per_s": round(g * 1e9 / 64 / 1e6, 1)}
            print(json.dumps(r), flush=True)
            rows.append(r)
    if args.out:
        Path(args.out).write_text("\n".join(json.dumps(r) for r in rows) + "\n")
    host.free()


if __name__ == "__main__":
    main()
