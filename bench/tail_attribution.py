#!/usr/bin/env python3
"""Attribute the ring-arrival -> scored latency tail of a deployed engine rank
 from a ``CCFD_SERVICE_TRACE`` dump (launch/engine_service.py).

Every traced micro-batch has host stamps (engine.cpp ``ccfd_batch_trace``, one monotonic clock):
arrival (oldest row committed to the pinned ring) -> submit (descriptor posted / launched) ->
landed (completion record in host memory) -> complete (retired).  Its latency splits into

* ``queued``  = submit - arrival: the row waited for the scoring thread to post it, and
* ``flight``  = landed - submit:  PCIe + kernel + completion record; where the persistent
  kernel stamped the batch (dev_start / dev_end, device clock) it splits further into
  ``device_exec`` = dev_end - dev_start (first item claimed -> last item done: the GPU's own
  time on the batch, which grows when several resident kernels share the device) and
  ``flight_other`` = the rest (doorbell + claim before the first item, completion record ->
  host after the last).  ``flight_other`` splits again, with the device clock aligned to the
  host's (``_device_split``), into ``device_start_wait`` (post -> first item claimed) and
  ``host_notice`` (last item done -> seen by the host); ``device_stall_windows`` lists the
  host-time windows in which the device started a batch >= 1 ms late or stopped it mid-run.

The queued part is cut against the scoring thread's own timeline: time INSIDE a native
``run()`` call (the thread was polling; a batch can still wait there for a free in-flight slot
or a partial batch for its flush deadline) versus time OUTSIDE it (the thread was in Python:
draining, commit snapshots, X2 ticks, or waiting for the GIL), and the outside time is further
split by what overlapped it: a scoring-thread task (X2 all-reduce tick / hot swap), a garbage
collection pause, a hand-off hold (scoring paused by back-pressure), or none of these (the
interpreter: GIL hand-over to another Python thread).

    python bench/tail_attribution.py gpurun_out/.../trace/rank0.npz [--out summary.json]
"""
from __future__ import annotations

import argparse
import json
from pathlib import Path

import numpy as np


def _intervals(a: np.ndarray):
    a = np.asarray(a, np.int64).reshape(-1, 2)
    return a[np.argsort(a[:, 0])] if len(a) else a


def _overlap(lo: int, hi: int, iv: np.ndarray) -> int:
    """Total length of [lo, hi) covered by the (sorted, possibly overlapping) intervals iv."""
    if hi <= lo or not len(iv):
        return 0
    i = max(0, int(np.searchsorted(iv[:, 0], lo, side="right")) - 1)
    tot, cur = 0, lo
    while i < len(iv) and iv[i, 0] < hi:
        a, b = max(iv[i, 0], cur), min(iv[i, 1], hi)
        if b > a:
            tot += b - a
            cur = b
        i += 1
    return int(tot)


def _gc_pauses(gc: np.ndarray) -> np.ndarray:
    out, t0 = [], None
    for t, phase, _g in np.asarray(gc).reshape(-1, 3):
        if phase == 0:
            t0 = t
        elif t0 is not None:
            out.append((t0, t))
            t0 = None
    return _intervals(np.array(out, np.int64))


def _held(held: np.ndarray, t_end: int) -> np.ndarray:
    out, t0 = [], None
    for t, h in np.asarray(held).reshape(-1, 2):
        if h and t0 is None:
            t0 = t
        elif not h and t0 is not None:
            out.append((t0, t))
            t0 = None
    if t0 is not None:
        out.append((t0, t_end))
    return _intervals(np.array(out, np.int64))


def _device_split(b: np.ndarray, window_ns: int = 500_000_000):
    """Per batch (post -> first item claimed, last item done -> seen in host memory), with the
    device clock aligned to the host's per ``window_ns`` window (drift): in each window the
    batch noticed fastest defines the offset (its notice = 0), so ``start`` and ``notice`` are
    exact up to that best-case notice latency (a few us)."""
    ts = b["t_submit"].astype(np.int64)
    tl = b["t_landed"].astype(np.int64)
    ds = b["dev_start"].astype(np.int64)
    de = b["dev_end"].astype(np.int64)
    w = (ts - ts.min()) // window_ns
    c = np.zeros(len(b), np.int64)
    for k in np.unique(w):
        m = w == k
        c[m] = (de[m] - tl[m]).max()
    return ds - c - ts, tl - (de - c)


def stall_windows(b: np.ndarray, start: np.ndarray, exe: np.ndarray, thr_ns: int = 1_000_000) -> dict:
    """Host-time windows in which a batch waited >= thr for the device to start it or was
    stopped mid-execution for >= thr: their lengths and spacing (a device time slice between
    several resident persistent kernels shows as fixed-length windows at a fixed period)."""
    big = (start >= thr_ns) | (exe >= thr_ns)
    iv = np.stack([b["t_submit"][big].astype(np.int64), b["t_landed"][big].astype(np.int64)], 1)
    iv = iv[np.argsort(iv[:, 0])] if len(iv) else iv
    merged = []
    for s_, e_ in iv:
        if merged and s_ <= merged[-1][1]:
            merged[-1][1] = max(merged[-1][1], e_)
        else:
            merged.append([s_, e_])
    m = np.array(merged, np.int64).reshape(-1, 2)
    if len(m) < 2:
        return {"windows": int(len(m))}
    ln = (m[:, 1] - m[:, 0]) / 1e6
    gap = np.diff(m[:, 0]) / 1e6
    return {"windows": int(len(m)), "length_ms": {"p50": round(float(np.median(ln)), 2), "max": round(float(ln.max()), 2)},
            "period_ms": {"p50": round(float(np.median(gap)), 1)},
            "share_of_time": round(float(ln.sum() / ((m[-1, 1] - m[0, 0]) / 1e6)), 3),
            "batches_started_late_ge_1ms": int((start >= thr_ns).sum()),
            "batches_stopped_mid_exec_ge_1ms": int((exe >= thr_ns).sum())}


def attribute(path: str, tail_q: float = 0.99) -> dict:
    d = np.load(path)
    b = d["batches"]
    b = b[b["t_arrival"] > 0]
    if not len(b):
        return {"trace": path, "batches": 0}
    native = bool(int(d["native"])) if "native" in d.files else False
    # the native serving thread (engine.cpp) is inside run() all the time
    runs = _intervals(np.array([[0, np.iinfo(np.int64).max]], np.int64)) if native else _intervals(d["runs"][:, :2])
    tasks = _intervals(d["tasks"])
    gcs = _gc_pauses(d["gc"])
    held = _held(d["held"], int(d["t_dump"]))
    total = (b["t_landed"] - b["t_arrival"]).astype(np.int64)
    queued = (b["t_submit"] - b["t_arrival"]).astype(np.int64)
    flight = (b["t_landed"] - b["t_submit"]).astype(np.int64)
    thr = np.quantile(total, tail_q)
    sel = np.nonzero(total >= thr)[0]
    dev = (b["dev_end"] - b["dev_start"]).astype(np.int64) if "dev_end" in b.dtype.names else np.zeros(len(b), np.int64)
    has_dev = dev > 0
    dstart = np.zeros(len(b), np.int64)
    notice = np.zeros(len(b), np.int64)
    if has_dev.all() and len(b) > 1:
        dstart, notice = _device_split(b)
    parts = {k: [] for k in ("in_run", "outside_run", "task", "gc", "held", "interpreter", "flight",
                             "device_exec", "flight_other", "device_start_wait", "host_notice")}
    for i in sel:
        lo, hi = int(b["t_arrival"][i]), int(b["t_submit"][i])
        inside = _overlap(lo, hi, runs)
        outside = max(0, (hi - lo) - inside)
        # outside-run time overlapped by each cause (a cause is charged only outside run())
        gaps = []
        if len(runs):
            k0 = max(0, int(np.searchsorted(runs[:, 1], lo)) - 1)
            cur = lo
            k = k0
            while k < len(runs) and runs[k, 0] < hi:
                if runs[k, 0] > cur:
                    gaps.append((cur, min(runs[k, 0], hi)))
                cur = max(cur, runs[k, 1])
                k += 1
            if cur < hi:
                gaps.append((cur, hi))
        else:
            gaps = [(lo, hi)]
        t_task = sum(_overlap(a, c, tasks) for a, c in gaps)
        t_gc = sum(_overlap(a, c, gcs) for a, c in gaps)
        t_held = sum(_overlap(a, c, held) for a, c in gaps)
        parts["in_run"].append(inside)
        parts["outside_run"].append(outside)
        parts["task"].append(t_task)
        parts["gc"].append(t_gc)
        parts["held"].append(t_held)
        parts["interpreter"].append(max(0, outside - t_task - t_gc - t_held))
        parts["flight"].append(int(flight[i]))
        de = int(dev[i]) if has_dev[i] else 0
        parts["device_exec"].append(de)
        parts["flight_other"].append(max(0, int(flight[i]) - de))
        parts["device_start_wait"].append(int(dstart[i]))
        parts["host_notice"].append(int(notice[i]))
    us = lambda v: round(float(v) / 1e3, 1)
    gaps_all = runs[1:, 0] - runs[:-1, 1] if len(runs) > 1 else np.zeros(0, np.int64)
    return {
        "trace": str(path), "batches": int(len(b)),
        "scoring_loop": "native C++ serving thread" if native else "Python scoring thread",
        "arrival_to_landed_us": {"p50": us(np.quantile(total, 0.5)), "p99": us(np.quantile(total, 0.99)),
                                 "max": us(total.max())},
        "queued_us": {"p50": us(np.quantile(queued, 0.5)), "p99": us(np.quantile(queued, 0.99))},
        "flight_us": {"p50": us(np.quantile(flight, 0.5)), "p99": us(np.quantile(flight, 0.99))},
        "device_exec_us": ({"p50": us(np.quantile(dev[has_dev], 0.5)), "p99": us(np.quantile(dev[has_dev], 0.99)),
                            "batches": int(has_dev.sum())} if has_dev.any() else None),
        # flight = device_start_wait (post -> first item claimed) + device_exec + host_notice
        "device_start_wait_us": ({"p50": us(np.quantile(dstart, 0.5)), "p99": us(np.quantile(dstart, 0.99))}
                                 if has_dev.all() and len(b) > 1 else None),
        "host_notice_us": ({"p50": us(np.quantile(notice, 0.5)), "p99": us(np.quantile(notice, 0.99))}
                           if has_dev.all() and len(b) > 1 else None),
        "device_stall_windows": stall_windows(b, dstart, dev) if has_dev.all() and len(b) > 1 else None,
        f"tail_batches_ge_p{int(tail_q * 100)}": int(len(sel)),
        "tail_mean_breakdown_us": {k: us(np.mean(v)) for k, v in parts.items()},
        "scoring_thread": {
            "run_calls": int(len(runs)),
            "gap_between_run_calls_us": {"p50": us(np.quantile(gaps_all, 0.5)) if len(gaps_all) else None,
                                         "p99": us(np.quantile(gaps_all, 0.99)) if len(gaps_all) else None,
                                         "max": us(gaps_all.max()) if len(gaps_all) else None},
            "tasks": int(len(tasks)), "task_ms_total": round(float((tasks[:, 1] - tasks[:, 0]).sum()) / 1e6, 1)
            if len(tasks) else 0.0,
            "gc_pauses": int(len(gcs)), "gc_ms_max": round(float((gcs[:, 1] - gcs[:, 0]).max()) / 1e6, 2)
            if len(gcs) else 0.0,
            "held_intervals": int(len(held))},
    }


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("traces", nargs="+")
    ap.add_argument("--tail-q", type=float, default=0.99)
    ap.add_argument("--out", default=None)
    a = ap.parse_args(argv)
    res = [attribute(t, a.tail_q) for t in a.traces]
    text = json.dumps(res if len(res) > 1 else res[0], indent=1)
    print(text)
    if a.out:
        Path(a.out).write_text(text + "\n")


if __name__ == "__main__":
    main()
