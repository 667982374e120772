"""Per-item phase table of the persistent G20 GBDT kernel.

Reads the device ring the experiment build dumps (`scripts/build_ab.py --name itrace --src
kernels/score_gbdt_g32_persist.hip --src engine/engine.cpp -D CCFD_EXP_ITEM_TRACE`, run with
`CCFD_LIB_PATH=.../ab/itrace.so CCFD_ITEM_TRACE_OUT=<prefix>`; one file per persistent engine
torn down, `<prefix>.<k>`).  Each record is one claimed item, stamped by its workgroup's thread 0
with the 100 MHz wall clock:

    claim      the work_next atomic, issue to value back (traces before round-5 pass L: issue only)
    wait_post  waiting until the item's micro-batch is posted (device mirror of the doorbell)
    desc       the per-item agent-scope acquire + the descriptor's atomic loads
    load       the first 64-row chunk's zero-copy load (issue -> data in registers)
    score      every chunk of the item (the next chunk's load overlaps the current one's trees)
    complete   counters, vmcnt drain of the outputs, system-scope release, ticket
    gap        from this item's ticket to the same workgroup's next claim

    python bench/experiments/item_trace.py gpurun_out/r5f/itrace.0 [--json out.json]
"""
import argparse
import json
import sys

import numpy as np

FIELDS = ("item", "wg", "t_claim", "t_claimed", "t_seen", "t_desc", "t_load", "t_scored", "t_done")
TICK_US = 0.01                                    # s_memrealtime: 100 MHz


ITEM_CAP, DB_CAP, DB_FIELDS = 1 << 17, 1 << 16, 8


def _ring(rec: np.ndarray, n: int) -> np.ndarray:
    cap = rec.shape[0]
    if n < cap:
        return rec[:n]
    k = n % cap                                   # ring: oldest first
    return np.concatenate([rec[k:], rec[:k]])


def load(path: str, doorbell: bool = False) -> np.ndarray:
    raw = np.fromfile(path, dtype=np.uint64)
    n = int(raw[0])
    item_words = ITEM_CAP * len(FIELDS)
    if raw.size in (1 + item_words, 2 + item_words + DB_CAP * DB_FIELDS):
        rec = raw[1:1 + item_words].reshape(-1, len(FIELDS))
    else:                                         # the first layout (pass r5f): no t_seen, no doorbell
        old = raw[1:].reshape(-1, len(FIELDS) - 1)
        rec = np.insert(old, FIELDS.index("t_seen"), old[:, FIELDS.index("t_claimed")], axis=1)
    if doorbell:
        if raw.size != 2 + item_words + DB_CAP * DB_FIELDS:
            return np.zeros((0, DB_FIELDS), np.int64)
        ndb = int(raw[1 + item_words])
        db = raw[2 + item_words:].reshape(-1, DB_FIELDS)
        return _ring(db, ndb).astype(np.int64)
    return _ring(rec, n).astype(np.int64)


def doorbell(db: np.ndarray, t_lo: int, t_hi: int) -> dict:
    """Doorbell cycles that found new postings, inside the items' time window: the poll's PCIe
    round trip, the descriptor copy + publish, batches delivered per cycle, and the interval
    between deliveries."""
    db = db[(db[:, 0] >= t_lo) & (db[:, 0] <= t_hi)]
    if len(db) < 2:
        return {"cycles": int(len(db))}
    rt = (db[:, 1] - db[:, 0]) * TICK_US
    cp = (db[:, 4] - db[:, 1]) * TICK_US
    nb = db[:, 2] - db[:, 3]
    iv = np.diff(db[:, 4]) * TICK_US
    q = lambda v: {"p50": round(float(np.median(v)), 2), "p90": round(float(np.percentile(v, 90)), 2),
                   "mean": round(float(v.mean()), 2)}
    return {"cycles": int(len(db)), "poll_round_trip_us": q(rt), "desc_copy_publish_us": q(cp),
            "batches_per_cycle": q(nb.astype(float)), "interval_between_deliveries_us": q(iv),
            "backlog_seen_ge2_share": round(float((nb >= 2).mean()), 3)}


def analyse(rec: np.ndarray, skip_frac: float = 0.02, items_per_batch: int = 0) -> dict:
    rec = rec[rec[:, FIELDS.index("t_done")] > 0]
    rec = rec[np.argsort(rec[:, 2], kind="stable")]
    lo = int(len(rec) * skip_frac)
    rec = rec[lo: len(rec) - lo]
    f = {k: rec[:, i] for i, k in enumerate(FIELDS)}
    ph = {
        "claim": f["t_claimed"] - f["t_claim"],
        "wait_post": f["t_seen"] - f["t_claimed"],
        "desc": f["t_desc"] - f["t_seen"],
        "load": f["t_load"] - f["t_desc"],
        "score": f["t_scored"] - f["t_load"],
        "complete": f["t_done"] - f["t_scored"],
    }
    # gap to the same workgroup's next claim
    gap = []
    for wg in np.unique(f["wg"]):
        s = rec[f["wg"] == wg]
        if len(s) > 1:
            gap.append(s[1:, 2] - s[:-1, FIELDS.index("t_done")])
    gap = np.concatenate(gap) if gap else np.zeros(1, np.int64)
    idle = gap >= int(100 / TICK_US)              # >= 100 us: the device had no posted work (phase ends)
    ph["gap"] = gap[~idle]
    total = f["t_done"] - f["t_claim"]
    span_us = (f["t_done"].max() - f["t_claim"].min()) * TICK_US
    wgs = len(np.unique(f["wg"]))
    out = {"items": int(len(rec)), "workgroups": wgs, "span_us": round(span_us, 1),
           "idle_gaps_ge_100us": int(idle.sum()), "idle_us_total": round(float(gap[idle].sum()) * TICK_US, 1),
           "items_per_s": round(len(rec) / (span_us * 1e-6), 1) if span_us > 0 else None,
           "item_us": {"p50": round(float(np.median(total)) * TICK_US, 2),
                       "mean": round(float(total.mean()) * TICK_US, 2)},
           "phases_us": {}}
    mean_total = float(total.mean() + ph["gap"].mean())
    for k, v in ph.items():
        v = v[v >= 0]
        if len(v) == 0:
            continue
        out["phases_us"][k] = {"p10": round(float(np.percentile(v, 10)) * TICK_US, 2),
                               "p50": round(float(np.median(v)) * TICK_US, 2),
                               "p90": round(float(np.percentile(v, 90)) * TICK_US, 2),
                               "p99": round(float(np.percentile(v, 99)) * TICK_US, 2),
                               "max": round(float(v.max()) * TICK_US, 2),
                               "mean": round(float(v.mean()) * TICK_US, 2),
                               "share_of_cycle": round(float(v.mean()) / mean_total, 3)}
    # per micro-batch (items_per_batch C): first claim -> last item done, and what its last item
    # spent: a batch completes -- and its ring slot is re-posted -- only behind its slowest item
    if items_per_batch:
        bidx = f["item"] // items_per_batch
        order = np.argsort(bidx, kind="stable")
        bs, starts = np.unique(bidx[order], return_index=True)
        spans, last_tot, last_wait = [], [], []
        for j in range(len(bs)):
            sl = order[starts[j]: starts[j + 1] if j + 1 < len(bs) else len(order)]
            if len(sl) != items_per_batch:
                continue                          # a batch only partly inside the ring
            k_last = sl[np.argmax(f["t_done"][sl])]
            spans.append(f["t_done"][sl].max() - f["t_claim"][sl].min())
            last_tot.append(f["t_done"][k_last] - f["t_claim"][k_last])
            last_wait.append(f["t_seen"][k_last] - f["t_claimed"][k_last])
        if spans:
            q = lambda v: {"p50": round(float(np.median(v)) * TICK_US, 1), "p99": round(float(np.percentile(v, 99)) * TICK_US, 1),
                           "max": round(float(np.max(v)) * TICK_US, 1)}
            out["batches"] = {"n": len(spans), "span_first_claim_to_last_done_us": q(np.array(spans)),
                              "last_item_total_us": q(np.array(last_tot)),
                              "last_item_wait_post_us": q(np.array(last_wait))}
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("paths", nargs="+")
    ap.add_argument("--json", default=None)
    ap.add_argument("--items-per-batch", type=int, default=128, help="micro-batch rows / item rows")
    a = ap.parse_args(argv)
    res = {}
    for p in a.paths:
        items = load(p)
        res[p] = analyse(items, items_per_batch=a.items_per_batch)
        db = load(p, doorbell=True)
        if len(db):
            res[p]["doorbell"] = doorbell(db, int(items[:, FIELDS.index("t_claim")].min()),
                                          int(items[:, FIELDS.index("t_done")].max()))
        r = res[p]
        print(f"{p}: {r['items']} items over {r['workgroups']} workgroups, {r['items_per_s']:.3g} items/s, "
              f"item p50 {r['item_us']['p50']} us")
        print(f"  {'phase':<10} {'p10':>8} {'p50':>8} {'p90':>8} {'mean':>8} {'share':>7}")
        for k, v in r["phases_us"].items():
            print(f"  {k:<10} {v['p10']:8.2f} {v['p50']:8.2f} {v['p90']:8.2f} {v['mean']:8.2f} {v['share_of_cycle']:7.1%}")
        if "batches" in r:
            print("  batches", json.dumps(r["batches"]))
        if "doorbell" in r:
            print("  doorbell", json.dumps(r["doorbell"]))
    if a.json:
        with open(a.json, "w") as fh:
            json.dump(res, fh, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
