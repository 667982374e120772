"""Summarise a rocprofv3 ``--kernel-trace`` database (rocpd SQLite, the rocprofv3 7.x default
output) into per-kernel statistics plus timeline facts the stats CSV does not give:
average kernel concurrency (sum of durations / busy span), per-queue idle gaps and the
number of distinct hardware queues used.

    python bench/kernel_timeline.py gpurun_out/prof9/run_results.db [--match score_] [--json out.json]
"""
from __future__ import annotations

import argparse
import json
import sqlite3
from collections import defaultdict

import numpy as np


def summarize(db: str, match: str = "") -> dict:
    c = sqlite3.connect(db)
    rows = c.execute("select name, start, end, queue_id, grid_x, workgroup_x from kernels order by start").fetchall()
    by = defaultdict(list)
    for name, s, e, q, gx, wx in rows:
        by[name].append((s, e, q, gx, wx))
    stats = []
    for name, v in by.items():
        d = np.array([e - s for s, e, *_ in v], np.float64)
        stats.append({"name": name[:120], "calls": len(v), "total_us": round(d.sum() / 1e3, 1),
                      "avg_us": round(d.mean() / 1e3, 2), "p50_us": round(float(np.median(d)) / 1e3, 2),
                      "min_us": round(d.min() / 1e3, 2), "max_us": round(d.max() / 1e3, 2),
                      "grid_x": v[0][3], "block_x": v[0][4]})
    stats.sort(key=lambda r: -r["total_us"])
    out = {"kernels": stats}
    sel = [r for r in rows if match in r[0]] if match else rows
    if sel:
        s0 = min(r[1] for r in sel)
        e1 = max(r[2] for r in sel)
        busy = sum(r[2] - r[1] for r in sel)
        # union of intervals = time with >= 1 kernel in flight
        iv = sorted((r[1], r[2]) for r in sel)
        union, cs, ce = 0, iv[0][0], iv[0][1]
        for s, e in iv[1:]:
            if s > ce:
                union += ce - cs
                cs, ce = s, e
            else:
                ce = max(ce, e)
        union += ce - cs
        qs = defaultdict(list)
        for r in sel:
            qs[r[3]].append((r[1], r[2]))
        gaps = []
        for q, v in qs.items():
            v.sort()
            gaps += [b[0] - a[1] for a, b in zip(v, v[1:])]
        g = np.array(gaps, np.float64) if gaps else np.zeros(1)
        out["timeline"] = {"match": match, "dispatches": len(sel), "span_us": round((e1 - s0) / 1e3, 1),
                           "busy_union_us": round(union / 1e3, 1),
                           "gpu_idle_frac": round(1 - union / max(1, e1 - s0), 4),
                           "avg_concurrency_when_busy": round(busy / max(1, union), 3),
                           "queues": len(qs), "queue_gap_p50_us": round(float(np.median(g)) / 1e3, 2),
                           "queue_gap_p90_us": round(float(np.percentile(g, 90)) / 1e3, 2)}
    return out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--match", default="score_")
    ap.add_argument("--json", default=None)
    a = ap.parse_args(argv)
    out = summarize(a.db, a.match)
    for r in out["kernels"][:8]:
        print(f'{r["calls"]:7d} {r["avg_us"]:9.2f} us avg {r["p50_us"]:8.2f} p50 {r["min_us"]:8.2f} min '
              f'grid {r["grid_x"]}x{r["block_x"]}  {r["name"][:70]}')
    if "timeline" in out:
        print(json.dumps(out["timeline"]))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)
    return out


if __name__ == "__main__":
    main()
