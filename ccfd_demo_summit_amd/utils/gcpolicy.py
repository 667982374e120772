"""Garbage-collector policy of the long-running Python services.

CPython's cyclic GC runs a full (generation 2) collection every ~700 x 10 x 10 allocations,
and a full collection walks every tracked object while holding the GIL.  A KIE server
holding ~10^5 process instances, or an engine rank whose router builds a dict per fraud-routed
row, then stalls for tens of milliseconds: the round-4 deployed-topology trace showed 886 GC
pauses of up to 98 ms on an engine rank, which were the entire arrival -> scored tail of the
Python scoring loop (profiles/r4/tail/).  These services create almost no reference cycles
(their state is dicts / deques of plain values), so:

* ``gc.freeze()`` after start-up moves everything allocated so far (imports, models, config)
  into the permanent generation -- never scanned again;
* young collections stay SMALL: generation 0 every ``gen0`` (10 000) allocations and
  generation 1 on every second one, so a pause scans at most a few 10^4 young objects
  (~7 ms), and survivors move on to generation 2;
* generation 2 (a full collection) needs ``gen2`` (10^6) generation-1 collections, i.e.
  practically never happens by itself.

Round 4 first used (50 000, 20, 1000): generation 1 then held up to 10^6 objects and a KIE
server starting ~10^4 fraud processes a second paused for up to 240 ms per collection
(``/rest/stats handoff_attribution.gc_pause_us``, profiles/r4/kie_handoff/): the TXB1
runs' scored -> process-started tail.  Measured on the KIE start + signal path: the old policy's
max pause 172 ms, (20 000, 1, 10^6) 13.6 ms, (10 000, 1, 10^6) 6.8 ms at the same throughput.

``CCFD_GC=default`` keeps CPython's defaults (A/B switch).
"""
from __future__ import annotations

import gc
import os


def tune_for_service(gen0: int = 10_000, gen1: int = 1, gen2: int = 1_000_000) -> str:
    """Apply the service GC policy (call once start-up is done); returns what was applied."""
    mode = os.environ.get("CCFD_GC", "service")
    if mode == "default":
        return "default"
    gc.collect()
    gc.freeze()
    gc.set_threshold(gen0, gen1, gen2)
    return f"frozen {gc.get_freeze_count()} objects, thresholds {gc.get_threshold()}"


def track_pauses(hist) -> None:
    """Record every cyclic-GC pass's duration (ns) into ``hist`` (utils.lathist.LatHist):
    the services' latency attribution names GC pauses instead of guessing them."""
    import time
    t0 = [0]

    def cb(phase, _info):
        if phase == "start":
            t0[0] = time.monotonic_ns()
        elif t0[0]:
            hist.add(time.monotonic_ns() - t0[0])
            t0[0] = 0
    gc.callbacks.append(cb)
