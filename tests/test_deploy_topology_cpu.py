"""bench/deploy_topology.py helpers (no GPU): Prometheus text parsing and the bucketed
quantile the harness reads Seldon latency with."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "bench"))


def test_metric_sum_and_bucket_quantile():
    import deploy_topology as dt
    text = "\n".join([
        "# TYPE transaction_outgoing_total counter",
        'transaction_outgoing_total{type="fraud"} 7.0',
        'transaction_outgoing_total{type="standard"} 993.0',
        "# TYPE lat_seconds histogram",
        'lat_seconds_bucket{status="200",le="0.0001"} 0.0',
        'lat_seconds_bucket{status="200",le="0.001"} 80.0',
        'lat_seconds_bucket{status="200",le="0.01"} 100.0',
        'lat_seconds_bucket{status="200",le="+Inf"} 100.0',
        'lat_seconds_count{status="200"} 100.0',
        'lat_seconds_sum{status="200"} 0.05',
    ]) + "\n"
    assert dt.metric_sum(text, "transaction_outgoing_total") == 1000.0
    assert dt.metric_sum(text, "transaction_outgoing_total", {"type": "fraud"}) == 7.0
    p50 = dt.hist_quantile_le(text, "lat_seconds", 0.5, {"status": "200"})
    assert 0.0001 < p50 < 0.001
    p99 = dt.hist_quantile_le(text, "lat_seconds", 0.99, {"status": "200"})
    assert 0.001 < p99 <= 0.01


def test_free_ports_are_bindable_and_contiguous():
    import socket
    import deploy_topology as dt
    base, = dt.free_ports(1, 3)
    for k in range(3):
        s = socket.socket()
        s.bind(("127.0.0.1", base + k))
        s.close()


def test_free_ports_never_repeat():
    import deploy_topology as dt
    a = dt.free_ports(1, 3)[0]
    b = dt.free_ports(4)
    c = dt.free_ports(1, 2)[0]
    used = {a, a + 1, a + 2, *b, c, c + 1}
    assert len(used) == 3 + 4 + 2
