"""Tracing helpers (SURVEY.md §5 tracing / profiling): the engine's per-batch stage trace
as a Chrome / Perfetto timeline."""
def test_batch_trace_events_tracks_and_device_alignment():
    """Engine per-batch stage trace -> Chrome events: four tracks, spans in order, device
    spans aligned so none ends after the host saw its completion record."""
    import numpy as np
    from ccfd_demo_summit_amd.ops._lib import BATCH_TRACE_DTYPE
    from ccfd_demo_summit_amd.utils.tracing import batch_trace_events
    tr = np.zeros(3, BATCH_TRACE_DTYPE)
    for i in range(3):
        base = 1_000_000 + i * 10_000
        tr[i] = (i, 0, 4096, base - 5_000 if i else 0, base, base + 40_000, base + 41_000,
                 7_000_000_000 + base + 2_000, 7_000_000_000 + base + 38_000 + i * 500, i, 0)
    ev = batch_trace_events(tr)
    names = {e["args"]["name"] for e in ev if e["ph"] == "M" and e["name"] == "thread_name"}
    assert names == {"queued", "in flight", "device", "hand-off"}
    spans = [e for e in ev if e["ph"] == "X"]
    assert len([e for e in spans if e["tid"] == 0]) == 2            # batch 0 had no ring arrival
    assert len([e for e in spans if e["tid"] == 2]) == 3
    for b in range(3):
        fl = next(e for e in spans if e["tid"] == 1 and e["name"] == f"batch {b}")
        dv = next(e for e in spans if e["tid"] == 2 and e["name"] == f"batch {b}")
        assert dv["ts"] + dv["dur"] <= fl["ts"] + fl["dur"] + 1e-9
        assert abs(dv["dur"] - (36_000 + b * 500) / 1e3) < 1e-9
    assert min(e["ts"] for e in spans) == 0.0
