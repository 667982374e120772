#!/usr/bin/env python3
"""GBDT ingest-binning microbench: ns per row of the G20 / G32 row encoders.

The G20 / G32 rows the GBDT kernels score are the `x_f > thr` half of tree evaluation done
at ingest (csrc/engine/binenc.h).  This measures, single-threaded and with T threads, the
branch-free SIMD encoder against the scalar binary-search encoder it replaced
(`ccfd_encode_g*_ref`), on a BASELINE-shaped table (oblivious GBDT 100 x 6, random init or
trained), and prints one JSON line.  Reference op: deploy/model/modelfull.json:37-44 (the
model's predict); BASELINE.json configs[3].

    python bench/encode_bench.py [--rows 1000000] [--threads 8] [--trained]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def ns_per_row(fn, args, n, reps=5):
    best = float("inf")
    for _ in range(reps):
        t0 = time.perf_counter()
        r = fn(*args)
        best = min(best, time.perf_counter() - t0)
        assert r == n, r
    return best / n * 1e9


def measure(rows: int = 1_000_000, threads: int = 8, trained: bool = False, seed: int = 0, bits: int = 5) -> dict:
    from ccfd_demo_summit_amd.data import generate
    from ccfd_demo_summit_amd.models.gbdt import ObliviousGBDT
    from ccfd_demo_summit_amd.ops._lib import lib
    L = lib()
    X, y = generate(rows, seed=seed)
    if trained:
        from ccfd_demo_summit_amd.train.trainer import train_oblivious_gbdt
        Xt, yt = generate(200_000, seed=seed + 1, fraud_rate=0.01)
        model, _ = train_oblivious_gbdt(Xt, yt, n_trees=100, depth=6, device="cpu", n_bins=32)
    else:
        model = ObliviousGBDT.random_init(100, 6, seed=seed, X_ref=X[:100_000])
    spec = model.bin_spec(bits=bits)
    rb = 20 if bits == 5 else 32
    out = np.zeros((rows, rb), np.uint8)
    am = np.zeros(rows, np.float32)
    flat, offs = spec.flat, spec.offsets          # keep the arrays alive while raw pointers are in use
    args = (X.ctypes.data, rows, 30, flat.ctypes.data, offs.ctypes.data, spec.stamp,
            out.ctypes.data, am.ctypes.data)
    simd = L.ccfd_encode_g20 if bits == 5 else L.ccfd_encode_g32
    ref = L.ccfd_encode_g20_ref if bits == 5 else L.ccfd_encode_g32_ref
    ns_ref = ns_per_row(ref, args, rows)
    ref_out = out.copy()
    ns_simd = ns_per_row(simd, args, rows)
    assert (out == ref_out).all(), "SIMD encoder disagrees with the scalar oracle"
    isa = {2: "avx512", 1: "avx2", 0: "scalar"}.get(int(L.ccfd_encode_isa(int(bits == 5))), "?")
    ns_avx2 = None
    if isa == "avx512":                       # the AVX2 path on the same host, for the record
        os.environ["CCFD_ENCODE_NO_AVX512"] = "1"
        try:
            out[:] = 0
            ns_avx2 = round(ns_per_row(simd, args, rows), 2)
            assert (out == ref_out).all(), "AVX2 encoder disagrees with the scalar oracle"
        finally:
            del os.environ["CCFD_ENCODE_NO_AVX512"]
    mt_args = args[:6] + (int(bits == 5), out.ctypes.data, am.ctypes.data, threads)
    ns_mt = ns_per_row(L.ccfd_encode_bins_mt, mt_args, rows)
    ne = np.diff(offs)
    return {"bench": "gbdt_ingest_encode", "row_format": spec.row_format, "rows": rows,
            "model": f"oblivious_gbdt_100x6_{'trained' if trained else 'random'}",
            "max_thresholds_per_feature": int(ne.max()), "mean_thresholds_per_feature": round(float(ne.mean()), 2),
            "ns_per_row_scalar_ref": round(ns_ref, 2), "ns_per_row_simd": round(ns_simd, 2),
            "isa": isa, "ns_per_row_avx2": ns_avx2,
            "speedup_1thread": round(ns_ref / ns_simd, 2),
            "threads": threads, "ns_per_row_simd_mt": round(ns_mt, 3),
            "rows_per_s_1thread": round(1e9 / ns_simd, 1), "rows_per_s_mt": round(1e9 / ns_mt, 1),
            "cpus_visible": len(os.sched_getaffinity(0))}


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--trained", action="store_true", help="bin table of a trained 100x6 ensemble (31-border cap)")
    ap.add_argument("--bits", type=int, default=5, choices=[5, 8])
    ap.add_argument("--out", default=None)
    a = ap.parse_args(argv)
    r = measure(a.rows, a.threads, a.trained, bits=a.bits)
    line = json.dumps(r)
    print(line, flush=True)
    if a.out:
        Path(a.out).write_text(line + "\n")


if __name__ == "__main__":
    main()
