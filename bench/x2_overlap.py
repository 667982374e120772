#!/usr/bin/env python3
"""X2 overlap evidence from a rocprofv3 kernel trace ("verify in rocprof
that [the X2 all-reduce] does not delay the scoring kernel").

Input: the ``*kernel_trace.csv`` of a ``rocprofv3 --kernel-trace --output-format csv`` run of
bench.py with ``CCFD_FORCE_PG=1`` (a real RCCL process group at world 1; add
``CCFD_X2_ONE_RANK_KERNEL=1`` so the one-rank reduction is a device kernel, see
parallel/dp.py).  Output: one JSON document --

* the persistent scoring kernel's dispatches (``persist_kernel``): count, queue, span;
* every other kernel: count, queues, duration, and how many ran entirely INSIDE a resident
  persistent-kernel window (= concurrently with scoring, on another hardware queue);
* the RCCL kernels among them (name matches nccl / rccl), with the same numbers.

    python bench/x2_overlap.py gpurun_out/r3a/x2 > profiles/r3/x2_overlap/summary.json
"""
from __future__ import annotations

import bisect
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def _col(header, *cands):
    low = {h.lower(): h for h in header}
    for c in cands:
        if c.lower() in low:
            return low[c.lower()]
    for h in header:
        if any(c.lower() in h.lower() for c in cands):
            return h
    return None


def load(path_or_dir: str):
    files = [path_or_dir] if os.path.isfile(path_or_dir) else \
        sorted(glob.glob(os.path.join(path_or_dir, "**", "*kernel_trace.csv"), recursive=True))
    rows = []
    for f in files:
        with open(f, newline="") as fh:
            rd = csv.DictReader(fh)
            h = rd.fieldnames or []
            cn, cs, ce = _col(h, "Kernel_Name"), _col(h, "Start_Timestamp"), _col(h, "End_Timestamp")
            cq, cst = _col(h, "Queue_Id"), _col(h, "Stream_Id")
            for r in rd:
                rows.append({"name": r[cn], "start": int(r[cs]), "end": int(r[ce]),
                             "queue": r.get(cq) if cq else None, "stream": r.get(cst) if cst else None})
    return rows, files


def short(name: str) -> str:
    """Demangled name without its trailing argument list (names like
    ``void (anonymous namespace)::oneRankReduce<...>(void*, ...)`` keep their scope)."""
    n = name.strip()
    if n.endswith(")"):
        depth = 0
        for i in range(len(n) - 1, -1, -1):
            depth += {")": 1, "(": -1}.get(n[i], 0)
            if depth == 0:
                n = n[:i]
                break
    return n[-140:]


RCCL_RE = re.compile(r"nccl|rccl|oneRankReduce", re.I)


def analyse(rows):
    persist = sorted((r for r in rows if "persist_kernel" in r["name"]), key=lambda r: r["start"])
    starts = [r["start"] for r in persist]

    def inside(r):
        i = bisect.bisect_right(starts, r["start"]) - 1
        return i >= 0 and persist[i]["end"] >= r["end"]
    by = defaultdict(lambda: {"count": 0, "inside_persist": 0, "queues": set(), "streams": set(),
                              "dur_ns": []})
    for r in rows:
        if "persist_kernel" in r["name"]:
            continue
        d = by[short(r["name"])]
        d["count"] += 1
        d["inside_persist"] += int(inside(r))
        d["queues"].add(r["queue"])
        d["streams"].add(r["stream"])
        d["dur_ns"].append(r["end"] - r["start"])
    out = {}
    for k, d in sorted(by.items(), key=lambda kv: -kv[1]["count"]):
        ds = sorted(d["dur_ns"])
        out[k] = {"count": d["count"], "inside_persist_window": d["inside_persist"],
                  "queues": sorted(x for x in d["queues"] if x is not None),
                  "streams": sorted(x for x in d["streams"] if x is not None),
                  "dur_ns_p50": ds[len(ds) // 2], "dur_ns_max": ds[-1],
                  "rccl": bool(RCCL_RE.search(k))}
    span = sum(r["end"] - r["start"] for r in persist)
    return {
        "persist_kernel": {"dispatches": len(persist), "resident_ns_total": span,
                           "queues": sorted({r["queue"] for r in persist if r["queue"] is not None}),
                           "longest_ns": max((r["end"] - r["start"] for r in persist), default=0)},
        "rccl_kernels": {k: v for k, v in out.items() if v["rccl"]},
        "other_kernels": {k: v for k, v in out.items() if not v["rccl"]},
    }


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    if not argv:
        raise SystemExit(__doc__)
    rows, files = load(argv[0])
    res = analyse(rows)
    res["trace_files"] = files
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
