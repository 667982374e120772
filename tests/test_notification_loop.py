"""Crash-safe notification loop (README.md:558-569,590,603-605):

* KIE keeps each CustomerNotification in an outbox (its fraud instance's journal record) until
  the broker acknowledged it; a restarted KIE re-publishes what is still pending;
* the notifier's customer is a pure function of (seed, transaction id), deduplicates by
  process id, and commits a consumed offset only once the reply for every message below it
  is acknowledged -- a SIGKILLed notifier re-answers what it had in flight, identically."""
import json
import time

import numpy as np

from ccfd_demo_summit_amd.ingest.producer import BatchingPublisher
from ccfd_demo_summit_amd.process import ProcessEngine
from ccfd_demo_summit_amd.process.notifier import NotificationService, encode_notification


def _starts(n, base=1000):
    return [{"transaction_id": base + i, "customer_id": i, "amount": 10.0 + i, "proba": 0.9} for i in range(n)]


def test_outbox_republishes_unacknowledged_notifications(tmp_path):
    j = str(tmp_path / "kie.jsonl")
    sent = []
    e = ProcessEngine(notification_timeout_s=60, journal_path=j, publish_notification=sent.append)
    ids = e.start_fraud_many(_starts(10))
    assert [m["process_id"] for m in sent] == ids
    e.mark_notified(ids[:6])                         # the broker acknowledged six of them
    e.close()                                        # ... and KIE dies
    r = ProcessEngine.recover(j, notification_timeout_s=60)
    pend = r.pending_notifications()
    assert sorted(m["process_id"] for m in pend) == sorted(ids[6:])
    assert {m["transaction_id"] for m in pend} == {1006, 1007, 1008, 1009}
    assert r.pending_notifications() == [] and r.notified_count == 6
    r.mark_notified([m["process_id"] for m in pend])
    r.close()
    r2 = ProcessEngine.recover(j, notification_timeout_s=60)
    assert r2.pending_notifications() == [] and r2.notified_count == 10
    # a completed instance whose notification was never acknowledged is still re-published
    r2.signal(ids[0], "customerResponse", True)
    r2.close()


def test_customer_is_deterministic_per_transaction_and_dedupes_by_process():
    a = NotificationService(lambda raw, key: None, p_reply=0.7, p_approve=0.5, mean_delay_s=0.5, seed=7)
    b = NotificationService(lambda raw, key: None, p_reply=0.7, p_approve=0.5, mean_delay_s=0.5, seed=7)
    c = NotificationService(lambda raw, key: None, p_reply=0.7, p_approve=0.5, mean_delay_s=0.5, seed=8)
    msgs = [{"transaction_id": 5000 + i, "process_id": i} for i in range(2000)]
    da = [a.decide(m) for m in msgs]
    # same seed, same transaction -> same reply and delay, whatever the process id
    assert da == [b.decide(dict(m, process_id=m["process_id"] * 3 + 1)) for m in msgs]
    assert da != [c.decide(m) for m in msgs]
    replies = sum(r for r, _a, _d in da)
    approves = sum(x for r, x, _d in da if r)
    assert abs(replies / 2000 - 0.7) < 0.05 and abs(approves / replies - 0.5) < 0.06
    assert abs(np.mean([d for r, _a, d in da if r]) - 0.5) < 0.08
    out = []
    ns = NotificationService(lambda raw, key: out.append(json.loads(raw)), p_reply=1.0, mean_delay_s=0.0, seed=1)
    for _ in range(3):                               # the outbox re-published it twice
        ns.handle(encode_notification({"transaction_id": 1, "process_id": 42}), now=0.0)
    ns.tick(now=1.0)
    assert len(out) == 1 and ns.duplicates == 2 and ns.sent == 1


def test_offsets_commit_only_behind_acknowledged_replies():
    toks = []
    ns = NotificationService(lambda raw, key, tok: toks.append(tok), p_reply=0.6, mean_delay_s=1.0, seed=3,
                             ack_async=True)
    msgs = [{"transaction_id": 70 + i, "process_id": i} for i in range(40)]
    replies = [o for o, m in enumerate(msgs) if ns.decide(m)[0]]
    for o, m in enumerate(msgs):
        ns.handle(encode_notification(m), now=0.0, offset=("n", 0, o))
    first = replies[0]
    assert ns.committable() == {("n", 0): first}           # no-reply messages before it are done
    ns.tick(now=1e6)                                        # every reply handed to the publisher
    assert len(toks) == len(replies) and ns.committable() == {("n", 0): first}
    toks.sort(key=lambda t: t[2])                           # (replies leave in due-time order)
    ns.on_published(toks[len(toks) // 2:])                  # the later offsets acknowledged first
    assert ns.committable() == {("n", 0): first}
    ns.on_published(toks[:1])
    assert ns.committable() == {("n", 0): toks[1][2]}
    ns.on_published(toks[1:len(toks) // 2])
    assert ns.committable() == {("n", 0): 40}


def test_kill_and_restart_both_sides_keeps_every_reply_once(tmp_path):
    """In-process rehearsal of the deployed check: KIE (journal + outbox) and the notifier over
    kafka-lite, both 'killed' mid-run (state dropped, consumer re-created from the committed
    offsets; KIE recovered from its journal), against a run without crashes: every notification
    answered once, every reply signalled once, identical outcomes."""
    from ccfd_demo_summit_amd.ingest.kafka_lite import KafkaLiteCluster
    from ccfd_demo_summit_amd.ingest.kafka_wire import KafkaBroker
    n = 300

    def run(crash: bool, d):
        cl = KafkaLiteCluster(1, default_partitions=2, data_dir=str(d / "kl")).start_in_thread()
        kb = KafkaBroker(cl.bootstrap, idempotent=True)
        for t in ("out", "resp"):
            kb.create_topic(t, 2)
        j = str(d / "kie.jsonl")
        state = {}

        def make_kie(recover):
            pub = BatchingPublisher(kb, "out", linger_s=0.001, on_sent=lambda t: state["eng"].mark_notified(t))
            kw = dict(notification_timeout_s=5.0, dmn_amount_threshold=100.0,
                      publish_notification=lambda m: pub.publish(encode_notification(m), token=m["process_id"]))
            eng = ProcessEngine.recover(j, **kw) if recover else ProcessEngine(journal_path=j, **kw)
            state["eng"], state["pub"] = eng, pub
            for m in eng.pending_notifications():
                pub.publish(encode_notification(m), token=m["process_id"])
            return eng

        def make_notifier():
            rpub = BatchingPublisher(kb, "resp", linger_s=0.001, on_sent=lambda t: state["ns"].on_published(t))
            ns = NotificationService(lambda raw, key, tok: rpub.publish(raw, token=tok), p_reply=0.8,
                                     mean_delay_s=0.05, seed=11, ack_async=True)
            state["ns"], state["rpub"] = ns, rpub
            return ns, kb.consumer("notification-service", ["out"])

        eng = make_kie(False)
        ns, cons = make_notifier()
        resp = kb.consumer("router-responses", ["resp"])
        signals = {"ok": 0, "stale": 0}

        def pump(t_s):
            t_end = time.monotonic() + t_s
            while time.monotonic() < t_end:
                for r in cons.poll(timeout=0.01, max_records=1000):
                    state["ns"].handle(r.value, offset=(r.topic, r.partition, r.offset))
                state["ns"].tick()
                offs = state["ns"].committable()
                if offs:
                    cons.commit(offs)
                for r in resp.poll(timeout=0.0, max_records=1000):
                    m = json.loads(r.value)
                    ok = state["eng"].signal(m["process_id"], "customerResponse", m["response"])
                    signals["ok" if ok else "stale"] += 1
                resp.commit()
                state["eng"].tick()
        for k in range(0, n, 50):
            eng.start_fraud_many(_starts(50, base=1000 + k))
            pump(0.05)
            if crash and k == 100:
                # KIE dies with notifications still unpublished; the notifier dies with replies
                # in its delay heap; both come back (KIE from its journal)
                state["pub"]._stop = True
                state["rpub"]._stop = True
                eng.close()
                eng = make_kie(True)
                ns, cons = make_notifier()
        t0 = time.monotonic()
        waiting = lambda: any(i.state.value == "waiting_customer" for i in state["eng"].instances.values())
        while waiting() and time.monotonic() - t0 < 30:
            pump(0.1)
        out = dict(eng.outcome_counts), signals, state["ns"].stats(), eng.notified_count, eng.outcome_digest
        # the digest is rebuilt from the journal: a recovered engine reports the same one
        assert ProcessEngine.recover(j, notification_timeout_s=5.0).outcome_digest == eng.outcome_digest
        state["pub"].close(1.0)
        state["rpub"].close(1.0)
        kb.close()
        cl.stop()
        return out
    (d1 := tmp_path / "a").mkdir()
    (d2 := tmp_path / "b").mkdir()
    oc_ref, sig_ref, _ns_ref, _, dg_ref = run(False, d1)
    oc, sig, _ns, notified, dg = run(True, d2)
    assert sum(oc_ref.values()) == n and oc == oc_ref, (oc, oc_ref)
    assert dg == dg_ref != 0                 # outcome for outcome, not only the totals
    assert sig["ok"] == sig_ref["ok"] == oc_ref["approved_by_customer"] + oc_ref["cancelled"]
    assert notified >= n
