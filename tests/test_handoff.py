"""Router -> KIE hand-off under a KIE outage (README.md:552,569):
the hand-off never blocks or raises on the scoring path, retries through a 5 s outage
(connection refused, then 5xx), and afterwards every fraud-routed transaction has been
started exactly once; offsets are committed only behind acknowledged hand-offs."""
import threading
import time

import numpy as np
import pytest

from ccfd_demo_summit_amd.ops._lib import FLAGGED_DTYPE
from ccfd_demo_summit_amd.process import ProcessEngine
from ccfd_demo_summit_amd.process.kie_server import KieClient
from ccfd_demo_summit_amd.router import Router, RuleSet
from ccfd_demo_summit_amd.router.handoff import KieHandoff
from tests.helpers.faulty_proxy import FaultyProxy
from tests.helpers.kie_thread import KieThread


def _flagged(ids):
    f = np.zeros(len(ids), np.dtype(FLAGGED_DTYPE))
    f["tx_id"] = ids
    f["customer"] = ids % 1000
    f["proba"] = 0.9
    f["amount"] = 42.0
    return f


@pytest.fixture()
def kie():
    procs = ProcessEngine(notification_timeout_s=1e9)
    k = KieThread(procs)
    px = FaultyProxy(k.port)
    yield procs, k, px
    px.close()
    k.close()


def test_kie_outage_never_blocks_and_starts_exactly_once(kie):
    procs, _, px = kie
    client = KieClient(px.url, timeout_s=1.0, pool_size=4)
    ho = KieHandoff(client, workers=3, max_batch=64, backoff_s=0.02, max_backoff_s=0.4)
    router = Router(RuleSet.threshold(0.5), client, handoff=ho)
    rng = np.random.default_rng(0)
    next_id = 1
    sent = []
    worst_call = 0.0
    t_start = time.monotonic()
    outage = (0.6, 5.6)                       # 2.5 s refused, then 2.5 s of 503s
    while time.monotonic() - t_start < 7.5:
        el = time.monotonic() - t_start
        want = "pass" if not outage[0] <= el < outage[1] else ("refuse" if el < outage[0] + 2.5 else "503")
        if px.mode != want:
            px.set_mode(want)
        n = int(rng.integers(1, 40))
        ids = np.arange(next_id, next_id + n, dtype=np.uint64)
        next_id += n
        sent.extend(ids.tolist())
        t0 = time.perf_counter()
        router.on_flagged(_flagged(ids), 4096)                 # must never block or raise
        worst_call = max(worst_call, time.perf_counter() - t0)
        time.sleep(0.01)
    assert worst_call < 0.05, worst_call
    assert ho.drain(30), ho.stats()
    st = ho.stats()
    assert st["retries"] > 0 and st["failed"] == 0 and st["depth"] == 0
    assert st["acked"] == st["submitted"] == len(sent)
    # every fraud-routed transaction started exactly once (re-sent batches were deduplicated)
    started = {inst.variables["transaction_id"] for inst in procs.instances.values()}
    assert started == set(sent)
    assert len(procs.instances) == len(sent)
    assert router.fraud_started == len(sent)
    ho.close()


def test_acked_seq_is_a_contiguous_prefix():
    """Out-of-order completion across workers: acked_seq only advances over a prefix."""
    gate = threading.Event()
    done = []

    class Sink:
        def start_fraud_many(self, items):
            if items[0]["transaction_id"] == 0:
                gate.wait(5)                       # the first batch is slow
            done.append(items[0]["transaction_id"])

        def start_fraud(self, v):
            self.start_fraud_many([v])

    ho = KieHandoff(Sink(), workers=3, max_batch=2)
    s0 = ho.submit_starts([{"transaction_id": 0}, {"transaction_id": 1}])
    s1 = ho.submit_starts([{"transaction_id": 2}, {"transaction_id": 3}])
    t0 = time.time()
    while 2 not in done and time.time() - t0 < 5:
        time.sleep(0.01)
    assert 2 in done and not ho.acked(s0) and not ho.acked(s1)
    gate.set()
    assert ho.drain(5) and ho.acked(s1)
    ho.close()


def test_full_queue_reports_backpressure():
    block = threading.Event()

    class Sink:
        def start_fraud_many(self, items):
            block.wait(5)

        def start_fraud(self, v):
            block.wait(5)
    ho = KieHandoff(Sink(), capacity=100, workers=1, max_batch=50)
    ho.submit_starts([{"transaction_id": i} for i in range(150)])
    assert ho.full() and not ho.has_room()
    block.set()
    assert ho.drain(5) and ho.has_room() and ho.depth() == 0
    ho.close()


def test_refused_without_dlq_is_held_not_acked():
    """a non-retryable answer must never be acked unsent (the engine would commit
    the offsets covering those fraud rows).  Without a DLQ the request is held and retried."""
    calls = []

    class Sink:
        def start_fraud_many(self, items):
            calls.append(len(items))
            raise ValueError("404 container not instantiated")
    ho = KieHandoff(Sink(), workers=1, backoff_s=0.01, max_backoff_s=0.05)
    seq = ho.submit_starts([{"transaction_id": 1}, {"transaction_id": 2}])
    assert not ho.drain(0.5)
    st = ho.stats()
    assert not ho.acked(seq) and st["refused"] == 1 and st["acked"] == 0 and st["depth"] == 2
    assert len(calls) >= 2                       # still being retried
    ho._stop = True


def test_refused_starts_go_to_the_dlq_then_replay_exactly_once(kie, tmp_path):
    """KIE answers 404 (unknown container): the refused starts are written
    to the durable DLQ BEFORE they are acked (so the offsets can be committed), counted in
    dead_lettered; replay against a healthy KIE starts each exactly once, a second replay
    starts nothing."""
    import requests
    from ccfd_demo_summit_amd.router.handoff import DeadLetterQueue
    procs, k, px = kie
    bad = KieClient(px.url, container_id="no-such-container", timeout_s=1.0)
    with pytest.raises(requests.HTTPError):
        bad.start_fraud_many([{"transaction_id": 1}, {"transaction_id": 2}])
    dlq = DeadLetterQueue(str(tmp_path / "handoff-dlq.jsonl"))
    ho = KieHandoff(bad, workers=2, max_batch=16, backoff_s=0.01, dlq=dlq)
    router = Router(RuleSet.threshold(0.5), bad, handoff=ho)
    ids = np.arange(100, 150, dtype=np.uint64)
    router.on_flagged(_flagged(ids), 4096)
    seq = router.last_handoff_seq
    assert ho.drain(10) and ho.acked(seq)
    st = ho.stats()
    assert st["dead_lettered"] == 50 and st["refused"] == 4 and st["failed"] == 4
    assert len(procs.instances) == 0
    pend = DeadLetterQueue(dlq.path).pending()           # durable: a fresh reader sees them
    assert sorted(v["transaction_id"] for e in pend for v in e["payload"]) == ids.tolist()
    good = KieClient(px.url, timeout_s=1.0)
    res = DeadLetterQueue(dlq.path).replay(good)
    assert res == {"replayed": 4, "failed": 0, "pending": 0}
    assert sorted(i.variables["transaction_id"] for i in procs.instances.values()) == ids.tolist()
    assert DeadLetterQueue(dlq.path).replay(good)["replayed"] == 0
    assert len(procs.instances) == 50 and procs.duplicates == 0
    ho.close()


def test_transient_classification():
    import requests
    from ccfd_demo_summit_amd.router.handoff import _transient

    def http(code):
        r = requests.Response()
        r.status_code = code
        return requests.HTTPError(response=r)
    assert _transient(requests.ConnectionError("refused")) and _transient(requests.Timeout("slow"))
    assert _transient(http(503)) and _transient(http(429)) and _transient(http(408))
    assert not _transient(http(404)) and not _transient(http(400))
    assert not _transient(requests.exceptions.JSONDecodeError("x", "doc", 0))   # non-JSON 200 body
    assert not _transient(requests.exceptions.InvalidURL("x"))
    assert not _transient(requests.exceptions.MissingSchema("x"))
    assert not _transient(ValueError("bad"))
    assert _transient(ConnectionRefusedError())


def test_signal_batch_falls_back_to_per_instance_route():
    """a KIE server without the signal/batch extension (404 / 405) must not drop
    every customer response: the hand-off switches to the per-instance signal route."""
    import requests
    got = []

    class Sink:
        def signal_many(self, items):
            r = requests.Response()
            r.status_code = 405
            raise requests.HTTPError(response=r)

        def signal(self, iid, name, payload):
            got.append((iid, name, payload))
            return True
    ho = KieHandoff(Sink(), workers=1)
    for i in range(5):
        ho.submit_signal(i, "customerResponse", True)
    assert ho.drain(5)
    st = ho.stats()
    assert st["signals_ok"] == 5 and st["refused"] == 0 and st["batch_signals"] is False
    assert sorted(g[0] for g in got) == list(range(5))
    ho.close()


def test_standard_starts_through_the_handoff_exactly_once(kie):
    """Router(standard_mode="process"): the engine's standard-routed rows start one standard
    process each (README.md:552) through the same acked hand-off, as column batches; a
    re-delivered batch (at-least-once) is deduplicated per transaction id at KIE."""
    procs, _, px = kie
    client = KieClient(px.url, timeout_s=2.0)
    ho = KieHandoff(client, workers=2, max_batch=1000, backoff_s=0.02)
    router = Router(RuleSet.threshold(0.5), client, standard_mode="process", handoff=ho)
    from ccfd_demo_summit_amd.ops._lib import SCORED_DTYPE
    std = np.zeros(3000, np.dtype(SCORED_DTYPE))
    std["tx_id"] = np.arange(10_000, 13_000)
    std["proba"] = 0.01
    std["amount"] = 7.5
    fl = _flagged(np.arange(1, 11, dtype=np.uint64))
    router.on_flagged(fl, 3010, standard=std)
    seq = router.last_handoff_seq
    router.on_flagged(fl[:0], 1000, standard=std[:1000])           # re-delivery of 1000 rows
    assert ho.drain(20) and ho.acked(seq)
    assert procs.standard_count == 3000 and procs.standard_duplicates == 1000
    assert len(procs._by_tx) == 10 and router.standard_started == 4000
    ho.close()


def test_signals_go_through_the_handoff(kie):
    procs, _, px = kie
    client = KieClient(px.url, timeout_s=1.0)
    ho = KieHandoff(client, workers=1, backoff_s=0.02)
    router = Router(RuleSet.threshold(0.5), client, handoff=ho)
    iid = procs.start_fraud({"transaction_id": 77, "customer_id": 1, "amount": 5.0, "proba": 0.9})
    px.set_mode("refuse")
    assert router.on_response(b'{"process_id": %d, "response": true}' % iid)   # queued, no raise
    time.sleep(0.3)
    px.set_mode("pass")
    assert ho.drain(10)
    assert procs.get(iid).outcome == "approved_by_customer"
    assert ho.stats()["signals_ok"] == 1 and ho.stats()["retries"] > 0
    ho.close()


def test_signals_are_coalesced_into_batch_requests(kie):
    """Customer responses arrive one per message; the hand-off sends the queued run of them
    as ONE `signal/batch` request (an HTTP request per signal capped the response loop)."""
    procs, _, px = kie
    client = KieClient(px.url, timeout_s=2.0)
    calls = []
    orig = client.signal_many

    def counting(items):
        calls.append(len(items))
        return orig(items)
    client.signal_many = counting
    ho = KieHandoff(client, workers=1, backoff_s=0.02)
    iids = [procs.start_fraud({"transaction_id": 1000 + i, "customer_id": i, "amount": 5.0, "proba": 0.9})
            for i in range(200)]
    px.set_mode("refuse")                        # let the signals pile up behind an outage
    for k, iid in enumerate(iids):
        ho.submit_signal(iid, "customerResponse", k % 2 == 0)
    ho.submit_signal(iids[0], "customerResponse", True)     # duplicate: stale, not an error
    time.sleep(0.2)
    px.set_mode("pass")
    assert ho.drain(10)
    st = ho.stats()
    assert st["signals_ok"] == 200 and st["signals_stale"] == 1 and st["failed"] == 0
    assert calls and all(c == 201 for c in calls), calls     # every attempt (retries too) is one batch
    assert sum(1 for i in iids if procs.get(i).outcome == "approved_by_customer") == 100
    ho.close()


def test_scored_to_started_attribution_on_both_sides(kie):
    """The scored -> process-started latency is split into where it is spent: the engine's
    hand-off queue wait and request time (KieHandoff.stats), and at the KIE server the
    request's arrival after scoring, the handler's own time and the event loop's lag
    (/rest/stats handoff_attribution)."""
    import json as _json
    import urllib.request

    from ccfd_demo_summit_amd.utils.lathist import LatHist
    procs, k, px = kie
    client = KieClient(px.url, timeout_s=2.0)
    ho = KieHandoff(client, workers=1, max_batch=64, backoff_s=0.02)
    router = Router(RuleSet.threshold(0.5), client, standard_mode="process", handoff=ho)
    from ccfd_demo_summit_amd.ops._lib import SCORED_DTYPE
    std = np.zeros(200, np.dtype(SCORED_DTYPE))
    std["tx_id"] = np.arange(50_000, 50_200)
    router.scored_ns = time.time_ns()
    router.on_flagged(_flagged(np.arange(1, 101, dtype=np.uint64)), 300, standard=std)
    assert ho.drain(20)
    st = ho.stats()
    assert st["queue_wait_us"]["n"] == st["request_us"]["n"] >= 2
    assert st["request_us"]["p50"] > 0
    time.sleep(0.2)                                 # a few timer ticks
    body = _json.loads(urllib.request.urlopen(f"http://127.0.0.1:{k.port}/rest/stats", timeout=5).read())
    att = body["handoff_attribution"]
    assert att["received_after_scored_us"]["n"] == 300          # every started row counted once
    assert att["start_handler_us"]["n"] >= 2 and att["timer_tick_us"]["n"] >= 1
    assert "journal_write_us" in att and "gc_pause_us" in att
    assert body["scored_to_started_us"]["n"] == 300
    # the histogram's interpolated quantiles stay inside the bucket of the values added
    h = LatHist()
    for v in (1000, 2000, 4000, 1_000_000):
        h.add(v)
    s = h.summary_us()
    assert s["n"] == 4 and 0.8 <= s["p50"] <= 2.5 and s["max"] == 1000.0
    ho.close()


def test_queued_standard_batches_are_coalesced():
    """Process mode hands off ~1e6 standard starts a second: batches queued behind a request in
    flight leave as ONE request (up to max_standard_batch rows), every seq still acked."""
    gate = threading.Event()
    calls = []

    class Sink:
        def start_standard_many(self, cols):
            gate.wait(5)
            calls.append(len(cols["transaction_id"]))
            return list(range(len(cols["transaction_id"])))
    ho = KieHandoff(Sink(), workers=1, max_standard_batch=5000)
    seqs = [ho.submit_standard({"transaction_id": np.arange(k * 1000, k * 1000 + 1000),
                                "proba": np.zeros(1000, np.float32)}) for k in range(12)]
    time.sleep(0.05)
    gate.set()
    assert ho.drain(10) and all(ho.acked(s) for s in seqs)
    assert sum(calls) == 12_000 and len(calls) <= 4 and max(calls) <= 5000
    assert ho.stats()["depth"] == 0
    ho.close()
