"""KIE scale-out (process/sharding.py): starts are routed by transaction-id
hash, instance and task ids encode their shard so signals and task completions reach the
owner, each shard has its own journal / hand-off queue / dead-letter journal, a misrouted
request is refused with 421, and a shard restarted from its journal keeps every start
exactly once."""
import numpy as np
import pytest
import requests

from ccfd_demo_summit_amd.ops._lib import FLAGGED_DTYPE, SCORED_DTYPE
from ccfd_demo_summit_amd.process import ProcessEngine
from ccfd_demo_summit_amd.process.kie_server import BASE, KieClient
from ccfd_demo_summit_amd.process.sharding import (ShardedKieClient, kie_urls, shard_from_env, shard_of_id,
                                                   shard_of_tx)
from ccfd_demo_summit_amd.router import Router, RuleSet
from ccfd_demo_summit_amd.router.handoff import DeadLetterQueue, ShardedHandoff
from tests.helpers.kie_thread import KieThread

K = 3


def test_tx_hash_is_even_deterministic_and_vectorised():
    # the producers' id ranges share their low 40 bits: (i + 1) << 40 | n
    tx = np.concatenate([((i + 1) << 40) + np.arange(20_000, dtype=np.int64) for i in range(3)])
    sh = shard_of_tx(tx, 4)
    counts = np.bincount(sh, minlength=4)
    assert counts.min() > 0.2 * len(tx) and counts.max() < 0.3 * len(tx)
    assert all(shard_of_tx(int(t), 4) == s for t, s in zip(tx[::997], sh[::997]))
    assert shard_of_tx(12345, 1) == 0 and shard_of_id(7, 3) == 1
    assert list(shard_of_id(np.array([3, 4, 5]), 3)) == [0, 1, 2]


def test_kie_urls_and_shard_identity(monkeypatch):
    assert kie_urls("http://a:1,http://b:2", 2) == ["http://a:1", "http://b:2"]
    assert kie_urls("http://ccd-service-{shard}.ccd-service:8090", 3)[2] == "http://ccd-service-2.ccd-service:8090"
    assert kie_urls("http://ccd-service:8090", 1) == ["http://ccd-service:8090"]
    with pytest.raises(ValueError):
        kie_urls("http://ccd-service:8090", 4)           # 4 shards, one reachable
    monkeypatch.delenv("CCFD_KIE_SHARD", raising=False)
    assert shard_from_env(None, "ccd-service-3") == 3 and shard_from_env(None, "kie") == 0
    assert shard_from_env(2, "ccd-service-3") == 2
    monkeypatch.setenv("CCFD_KIE_SHARD", "1")
    assert shard_from_env(None, "ccd-service-3") == 1


def test_engine_ids_encode_the_shard_and_survive_recovery(tmp_path):
    j = str(tmp_path / "s1.jsonl")
    e = ProcessEngine(notification_timeout_s=0.0, dmn_amount_threshold=0.0, journal_path=j, shard=1, shards=K)
    ids = e.start_standard_many({"transaction_id": np.arange(100, 110, dtype=np.int64)})
    f = e.start_fraud({"transaction_id": 5, "amount": 500.0, "proba": 0.99})
    assert all(i % K == 1 for i in ids) and f % K == 1 and len(set(ids) | {f}) == 11
    e.tick(now=e.clock() + 1.0)                          # timer -> DMN -> user task
    (t,) = e.list_tasks()
    assert t.id % K == 1 and t.instance_id == f
    e.close()
    r = ProcessEngine.recover(j, notification_timeout_s=0.0, shard=1, shards=K)
    again = r.start_standard_many({"transaction_id": np.arange(105, 112, dtype=np.int64)})
    assert again[:5] == ids[5:] and all(i % K == 1 for i in again)
    assert len(set(again[5:]) & (set(ids) | {f})) == 0          # new ids never reuse old ones
    assert r.standard_count == 12 and r.standard_duplicates == 5 and r.fraud_count == 1
    assert r.tasks[t.id].instance_id == f
    r.close()


@pytest.fixture()
def tier(tmp_path):
    engines = [ProcessEngine(notification_timeout_s=1e9, journal_path=str(tmp_path / f"kie{k}.jsonl"),
                             shard=k, shards=K) for k in range(K)]
    servers = [KieThread(e) for e in engines]
    urls = ",".join(f"http://127.0.0.1:{s.port}" for s in servers)
    yield engines, servers, urls
    for s in servers:
        s.close()


def _flagged(ids):
    f = np.zeros(len(ids), np.dtype(FLAGGED_DTYPE))
    f["tx_id"] = ids
    f["customer"] = ids % 1000
    f["proba"] = 0.9
    f["amount"] = 420.0
    return f


def test_sharded_tier_routes_starts_signals_and_tasks(tier, tmp_path):
    engines, servers, urls = tier
    clients = [KieClient(u, timeout_s=5.0) for u in kie_urls(urls, K)]
    sk = ShardedKieClient(clients)
    dlqs = [DeadLetterQueue(str(tmp_path / f"dlq.shard{k}.jsonl")) for k in range(K)]
    ho = ShardedHandoff(clients, dlqs, workers=2, max_batch=512, backoff_s=0.02)
    router = Router(RuleSet.threshold(0.5), sk, standard_mode="process", handoff=ho)
    fraud_tx = np.arange(1, 61, dtype=np.uint64) + np.uint64(1 << 40)
    std = np.zeros(5000, np.dtype(SCORED_DTYPE))
    std["tx_id"] = np.arange(5000, dtype=np.uint64) + np.uint64(2 << 40)
    std["proba"] = 0.01
    std["amount"] = 3.0
    router.on_flagged(_flagged(fraud_tx), 5060, standard=std)
    g1 = router.last_handoff_seq
    router.on_flagged(_flagged(fraud_tx[:10]), 1010, standard=std[:1000])     # re-delivery
    g2 = router.last_handoff_seq
    assert g2 > g1 and ho.drain(20) and ho.acked(g2) and ho.acked(g1)
    # every transaction started exactly once, on the shard its id hashes to
    for k, e in enumerate(engines):
        mine_f = {int(t) for t in fraud_tx if shard_of_tx(int(t), K) == k}
        assert set(e._by_tx) == mine_f
        assert all(i % K == k for i in e.instances)
        assert e.standard_count == int((shard_of_tx(std["tx_id"].astype(np.int64), K) == k).sum())
    assert sum(e.standard_count for e in engines) == 5000 and sum(e.fraud_count for e in engines) == 60
    assert sum(e.standard_duplicates for e in engines) == 1000 and sum(e.duplicates for e in engines) == 10
    st = ho.stats()
    assert st["shards"] == K and st["acked"] == st["submitted"] and st["dead_lettered"] == 0
    # customer responses: the signal carries only the process id and reaches its owner
    iids = [iid for e in engines for iid, inst in e.instances.items() if inst.process_id == "fraud"]
    for n, iid in enumerate(sorted(iids)[:30]):
        router.on_response({"process_id": iid, "response": n % 2 == 0})
    g3 = router.last_handoff_seq
    assert ho.drain(10) and ho.acked(g3)
    oc = {k: sum(e.outcome_counts[k] for e in engines) for k in ("approved_by_customer", "cancelled")}
    assert oc == {"approved_by_customer": 15, "cancelled": 15}
    # user tasks: timers fire on every shard; a completion by task id reaches the owner
    for e in engines:
        e.timeout = 0.0
        for inst in e.instances.values():
            if inst.state.value == "waiting_customer":
                inst.timer_due = 0.0
                import heapq
                heapq.heappush(e._timers, (0.0, inst.id))
        e.tick(now=1e12)
    tasks = [(t.id, k) for k, e in enumerate(engines) for t in e.list_tasks()]
    assert tasks and all(tid % K == k for tid, k in tasks)
    for tid, k in tasks:
        r = requests.put(f"{urls.split(',')[shard_of_id(tid, K)]}{BASE}/containers/ccd-fraud-kjar/tasks/{tid}"
                         "/states/completed", json={"outcome": "approved"}, timeout=5)
        assert r.status_code == 201
    assert all(not e.list_tasks() for e in engines)
    # a misrouted request is refused (421), never served by the wrong shard
    tid, k = tasks[0]
    wrong = urls.split(",")[(k + 1) % K]
    r = requests.get(f"{wrong}{BASE}/containers/ccd-fraud-kjar/tasks/{tid}", timeout=5)
    assert r.status_code == 421
    bad_tx = next(int(t) for t in range(10**6, 10**6 + 50) if shard_of_tx(t, K) != 0)
    r = requests.post(f"{urls.split(',')[0]}{BASE}/containers/ccd-fraud-kjar/processes/"
                      "ccd-fraud-kjar.StandardProcess/instances", json={"transaction_id": bad_tx}, timeout=5)
    assert r.status_code == 421 and engines[0].standard_count == sum(
        1 for t in std["tx_id"].astype(np.int64) if shard_of_tx(int(t), K) == 0)
    ho.close()


def test_a_restarted_shard_keeps_starts_exactly_once(tier, tmp_path):
    engines, servers, urls = tier
    clients = [KieClient(u, timeout_s=5.0) for u in kie_urls(urls, K)]
    sk = ShardedKieClient(clients)
    cols = {"transaction_id": np.arange(30_000, dtype=np.int64) + (3 << 40),
            "amount": np.full(30_000, 2.0, np.float32), "proba": np.full(30_000, 0.1, np.float32)}
    sk.start_standard_many(cols)
    # shard 2 crashes and comes back from its journal; the whole batch is re-delivered
    servers[2].close()
    engines[2].close()
    rec = ProcessEngine.recover(str(tmp_path / "kie2.jsonl"), notification_timeout_s=1e9, shard=2, shards=K)
    servers[2] = KieThread(rec)
    clients[2] = KieClient(f"http://127.0.0.1:{servers[2].port}", timeout_s=5.0)
    sk = ShardedKieClient(clients)
    ids = sk.start_standard_many(cols)
    engines[2] = rec
    assert sum(e.standard_count for e in engines) == 30_000
    assert sum(e.standard_duplicates for e in engines) == 30_000
    assert len(set(ids)) == 30_000 and all(i % K == shard_of_tx(int(t), K) for i, t in
                                           zip(ids[::101], cols["transaction_id"][::101]))
