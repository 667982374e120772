"""Native JSON-per-transaction ingest throughput (csrc/engine/ingest.cpp), CPU only.

The reference producer publishes one transaction per Kafka message (README.md:547-548) and
the router extracts the model features from it (README.md:549).  This times
``ccfd_parse_json_batch`` / ``ccfd_parse_json_batch_w64`` on messages shaped like that
(named columns Time, V1..V28, Amount plus id / customer_id, 6 significant digits) and
reports rows/s per host thread.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def messages(n: int, seed: int = 0):
    from ccfd_demo_summit_amd.contracts import FEATURE_NAMES
    from ccfd_demo_summit_amd.data import generate
    X, _ = generate(n, seed=seed)
    msgs = [(f'{{"id":{i},"customer_id":{i % 100000},' +
             ",".join(f'"{k}":{float(v):.6g}' for k, v in zip(FEATURE_NAMES, X[i])) + "}").encode()
            for i in range(n)]
    return msgs, X


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--rows", type=int, default=200_000)
    ap.add_argument("--repeat", type=int, default=5)
    ap.add_argument("--out", default=None)
    args = ap.parse_args(argv)
    from ccfd_demo_summit_amd.ops._lib import lib
    L = lib()
    msgs, X = messages(args.rows)
    buf = b"".join(msgs)
    off = np.zeros(len(msgs) + 1, np.int64)
    off[1:] = np.cumsum([len(m) for m in msgs])
    n = len(msgs)
    f = np.zeros((n, 30), np.float32)
    rows = np.zeros((n, 64), np.uint8)
    ids = np.zeros(n, np.uint64)
    cu = np.zeros(n, np.uint32)
    res = {"rows": n, "bytes_per_msg": round(len(buf) / n, 1)}
    for name, fn, out in (("f32", L.ccfd_parse_json_batch, f), ("w64", L.ccfd_parse_json_batch_w64, rows)):
        best = 1e9
        for _ in range(args.repeat):
            t0 = time.perf_counter()
            rc = fn(buf, off.ctypes.data, n, out.ctypes.data, ids.ctypes.data, cu.ctypes.data)
            best = min(best, time.perf_counter() - t0)
            assert rc == n, rc
        res[f"{name}_rows_per_s"] = round(n / best, 1)
        res[f"{name}_MBps"] = round(len(buf) / best / 1e6, 1)
    ref = np.array([[float(f"{v:.6g}") for v in row] for row in X[:1000]], np.float32)
    res["max_abs_err_vs_python_float"] = float(np.abs(f[:1000] - ref).max())
    line = json.dumps(res)
    print(line)
    if args.out:
        Path(args.out).write_text(line + "\n")


if __name__ == "__main__":
    main()
