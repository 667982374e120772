"""Business-process state machine: all terminal outcomes, DMN, prediction-service
confidence rule, journal recovery, duplicate signals."""
import numpy as np
import pytest

from ccfd_demo_summit_amd.contracts.outcomes import Outcome
from ccfd_demo_summit_amd.metrics import KieMetrics
from ccfd_demo_summit_amd.process import (Decision, NotificationService, PredictionService, ProcessEngine,
                                          State, investigation_decision, investigation_decision_batch)


class Clock:
    def __init__(self):
        self.t = 0.0

    def __call__(self):
        return self.t


def _engine(conf=1.0, **kw):
    clock = Clock()
    sent = []
    m = KieMetrics()
    eng = ProcessEngine(notification_timeout_s=10.0, dmn_probability_threshold=0.75, dmn_amount_threshold=100.0,
                        publish_notification=sent.append, kie_metrics=m,
                        prediction=PredictionService(conf), clock=clock, **kw)
    return eng, clock, sent, m


def _hist_count(h):
    return h._sum.get(), sum(b.get() for b in h._buckets)


def test_dmn():
    assert investigation_decision(0.5, 50, 0.75, 100) == Decision.APPROVE
    assert investigation_decision(0.9, 50, 0.75, 100) == Decision.INVESTIGATE
    assert investigation_decision(0.5, 500, 0.75, 100) == Decision.INVESTIGATE
    np.testing.assert_array_equal(investigation_decision_batch([0.5, 0.9, 0.5], [50, 50, 500], 0.75, 100),
                                  [False, True, True])


def test_customer_approves_and_rejects():
    eng, clock, sent, m = _engine()
    a = eng.start_fraud({"transaction_id": 1, "customer_id": 11, "amount": 20.0, "proba": 0.9})
    b = eng.start_fraud({"transaction_id": 2, "customer_id": 12, "amount": 30.0, "proba": 0.9})
    assert [s["process_id"] for s in sent] == [a, b]
    assert sent[0]["customer_id"] == 11 and sent[0]["transaction_id"] == 1
    assert eng.signal(a, "customerResponse", True)
    assert eng.signal(b, "customerResponse", "false")
    assert eng.get(a).outcome == Outcome.APPROVED_BY_CUSTOMER.value
    assert eng.get(b).outcome == Outcome.CANCELLED.value
    assert _hist_count(m.approved) == (20.0, 1)
    assert _hist_count(m.rejected) == (30.0, 1)
    # duplicate / late signal is ignored (at-least-once delivery)
    assert not eng.signal(a, "customerResponse", False)
    assert eng.get(a).outcome == Outcome.APPROVED_BY_CUSTOMER.value
    # timers of completed instances never fire
    clock.t = 100
    assert eng.tick() == 0


def test_timer_dmn_low_amount_and_investigation():
    eng, clock, sent, m = _engine(conf=1.0)
    low = eng.start_fraud({"transaction_id": 1, "amount": 20.0, "proba": 0.6})
    big = eng.start_fraud({"transaction_id": 2, "amount": 5000.0, "proba": 0.6})
    clock.t = 9.9
    assert eng.tick() == 0
    clock.t = 10.0
    assert eng.tick() == 2
    assert eng.get(low).outcome == Outcome.APPROVED_LOW_AMOUNT.value
    inst = eng.get(big)
    assert inst.state == State.USER_TASK
    tasks = eng.list_tasks()
    assert len(tasks) == 1 and tasks[0].instance_id == big
    # confidence threshold 1.0 (reference default): never auto-closed, outcome pre-filled
    assert tasks[0].suggested_outcome in ("approved", "rejected") and tasks[0].status == "Ready"
    assert _hist_count(m.approved_low) == (20.0, 1)
    assert _hist_count(m.investigation) == (5000.0, 1)
    # a signal arriving after the timer is stale
    assert not eng.signal(big, "customerResponse", True)
    assert eng.complete_task(tasks[0].id, "rejected")
    assert eng.get(big).outcome == Outcome.INVESTIGATION_CLOSED_FRAUD.value
    assert eng.prediction.training[-1]["outputs"] == {"outcome": "rejected"}


def test_prediction_service_auto_closes_above_threshold():
    eng, clock, _, _ = _engine(conf=0.5)
    iid = eng.start_fraud({"transaction_id": 3, "amount": 20000.0, "proba": 0.99})
    clock.t = 11
    eng.tick()
    inst = eng.get(iid)
    assert inst.state == State.COMPLETED
    assert inst.outcome == Outcome.INVESTIGATION_CLOSED_FRAUD.value
    assert eng.tasks[inst.task_id].completed_by == "prediction-service"


def test_prediction_service_rule():
    ps = PredictionService(0.8)
    out = ps.predict({"proba": 0.99, "amount": 20000})
    assert out.outcome == "rejected" and out.confidence > 0.8 and ps.should_auto_complete(out)
    out2 = PredictionService(1.0).predict({"proba": 0.99, "amount": 20000})
    assert not PredictionService(1.0).should_auto_complete(out2)


def test_standard_process():
    eng, *_ = _engine()
    iid = eng.start("ccd-fraud-kjar.standard", {"transaction_id": 9})
    assert eng.outcome_counts[Outcome.STANDARD.value] == 1 and iid == 1


def test_journal_recovery(tmp_path):
    j = str(tmp_path / "bp.jsonl")
    eng, clock, _, _ = _engine(journal_path=j)
    a = eng.start_fraud({"transaction_id": 1, "amount": 20.0, "proba": 0.9})
    b = eng.start_fraud({"transaction_id": 2, "amount": 5000.0, "proba": 0.9})
    eng.signal(a, "customerResponse", True)
    eng.close()
    clock2 = Clock()
    rec = ProcessEngine.recover(j, notification_timeout_s=10.0, clock=clock2)
    assert rec.get(a).outcome == Outcome.APPROVED_BY_CUSTOMER.value
    assert rec.get(b).state == State.WAITING_CUSTOMER
    clock2.t = 20
    assert rec.tick() == 1
    assert rec.get(b).state == State.USER_TASK
    c = rec.start_fraud({"transaction_id": 3, "amount": 1.0, "proba": 0.9})
    assert c > b
    rec.close()


def test_notifier_deterministic():
    def run(seed):
        out = []
        clock = Clock()
        ns = NotificationService(lambda raw, key: out.append(raw), p_reply=0.7, p_approve=0.5,
                                 mean_delay_s=1.0, seed=seed, clock=clock)
        import json
        for i in range(200):
            ns.handle(json.dumps({"customer_id": i, "transaction_id": i, "process_id": i}).encode())
        clock.t = 1e9
        ns.tick()
        return out, ns
    o1, ns1 = run(3)
    o2, _ = run(3)
    assert o1 == o2
    assert ns1.sent == 200 and ns1.replied + ns1.no_reply == 200
    assert 100 < ns1.replied < 180


def test_journal_recovery_survives_a_torn_last_line(tmp_path):
    """A KIE killed mid-write (SIGKILL) leaves a partial last journal line; recovery skips it
    and keeps the per-transaction dedupe index, so re-sent fraud starts are not doubled."""
    from ccfd_demo_summit_amd.process import ProcessEngine
    j = str(tmp_path / "j.jsonl")
    e = ProcessEngine(notification_timeout_s=60, journal_path=j)
    ids = [e.start_fraud({"transaction_id": t, "customer_id": 1, "amount": 5.0, "proba": 0.9}) for t in range(10)]
    e.close()
    with open(j, "a") as f:
        f.write('{"instance": {"id": 99, "process_id": "fr')           # torn write
    r = ProcessEngine.recover(j, notification_timeout_s=60)
    assert sorted(r.instances) == sorted(ids)
    assert r.start_fraud({"transaction_id": 3, "customer_id": 1, "amount": 5.0, "proba": 0.9}) == ids[3]
    assert r.duplicates == 1
    r.start_fraud({"transaction_id": 50, "customer_id": 1, "amount": 5.0, "proba": 0.9})
    r.close()
    r2 = ProcessEngine.recover(j, notification_timeout_s=60)        # the record after the torn line survives
    assert len(r2.instances) == 11 and 50 in r2._by_tx


def test_standard_batches_idempotent_and_recovered(tmp_path):
    """start_standard_many (the engine's standard-route hand-off): one process per transaction
    id -- within a batch, across re-delivered batches, and across a KIE restart from its
    journal; numpy columns are accepted."""
    import numpy as np
    from ccfd_demo_summit_amd.process import ProcessEngine
    j = str(tmp_path / "kie.jsonl")
    e = ProcessEngine(notification_timeout_s=60, journal_path=j)
    ids1 = e.start_standard_many({"transaction_id": np.array([10, 11, 12, 11], np.int64),
                                  "proba": np.array([0.1, 0.2, 0.3, 0.2], np.float32)})
    assert ids1[1] == ids1[3] and len(set(ids1)) == 3
    ids2 = e.start_standard_many([{"transaction_id": 12}, {"transaction_id": 13}])
    assert ids2[0] == ids1[2] and ids2[1] not in ids1
    f = e.start_fraud({"transaction_id": 99, "amount": 5.0, "proba": 0.9})
    assert e.standard_count == 4 and e.standard_duplicates == 2
    e.close()
    r = ProcessEngine.recover(j, notification_timeout_s=60)
    assert r.standard_count == 4 and r.outcome_counts["standard"] == 4
    again = r.start_standard_many({"transaction_id": [10, 13, 14]})
    assert again[:2] == [ids1[0], ids2[1]] and r.standard_count == 5
    assert again[2] > max(ids1 + ids2 + [f])          # fresh ids never collide after recovery
    r.close()


def test_start_fraud_many_matches_one_by_one_starts(tmp_path):
    """The batched fraud start (KIE instances/batch, the in-process router sink) has the
    per-transaction semantics of start_fraud: a duplicate inside the batch or from an earlier
    one returns the existing instance and publishes nothing; one journal record and one
    notification per new instance; the journal recovers the batch (timers included)."""
    from ccfd_demo_summit_amd.process.engine import ProcessEngine
    j = str(tmp_path / "j.jsonl")
    sent = []
    e = ProcessEngine(notification_timeout_s=30, journal_path=j, publish_notification=sent.append,
                      clock=lambda: 100.0)
    first = e.start_fraud({"transaction_id": 7, "customer_id": 1, "amount": 5.0, "proba": 0.9})
    items = [{"transaction_id": t, "customer_id": t % 3, "amount": float(t), "proba": 0.8, "scored_ns": 1}
             for t in (1, 2, 7, 3, 2)]
    ids = e.start_fraud_many(items)
    assert ids[2] == first and ids[4] == ids[1] and len(set(ids)) == 4
    assert e.duplicates == 2 and len(e._by_tx) == 4
    assert [m["transaction_id"] for m in sent] == [7, 1, 2, 3]
    assert [m["process_id"] for m in sent[1:]] == [ids[0], ids[1], ids[3]]
    cols = e.start_fraud_many({"transaction_id": [4, 1], "customer_id": [0, 0], "amount": [1.0, 1.0],
                               "proba": [0.7, 0.7]})
    assert cols[1] == ids[0] and len(e._by_tx) == 5
    e.close()
    r = ProcessEngine.recover(j, notification_timeout_s=30, clock=lambda: 100.0)
    assert sorted(r._by_tx) == [1, 2, 3, 4, 7]
    assert r.tick(now=131.0) == 5                      # every recovered timer fires once
