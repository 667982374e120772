"""Standard-start idempotency gated by the engine's committed offsets, and the by-transaction
audit query (reference README.md:552 -- every transaction starts a
process).

A count window alone loses idempotency when one KIE shard is down long enough: the engine's
commit waits behind that shard while the live shards keep admitting, so a replay after an
engine crash can reach past their windows.  Here a standard batch's transaction ids stay until
the engine reports its commits past the batch's marks, however many other ids arrive.
"""
import asyncio
import os

import numpy as np
import pytest
from aiohttp.test_utils import TestClient, TestServer

from ccfd_demo_summit_amd.process.dedupe import DedupeFull, DedupeIndex
from ccfd_demo_summit_amd.process.engine import ProcessEngine
from ccfd_demo_summit_amd.process.kie_server import BASE, KieServer, encode_columns
from ccfd_demo_summit_amd.process.sharding import shard_of_tx


def _batch(tx, part, mark, proba=None):
    tx = np.asarray(tx, np.int64)
    cols = {"transaction_id": tx, "customer_id": np.zeros(len(tx), np.int64),
            "amount": np.full(len(tx), 2.5, np.float32),
            "proba": (np.full(len(tx), 0.01, np.float32) if proba is None else np.asarray(proba, np.float32))}
    if part is not None:
        cols["kafka_partition"] = np.full(len(tx), part, np.int64)
        cols["commit_mark"] = np.full(len(tx), mark, np.int64)
    return cols


def test_native_gated_index_refuses_and_evicts():
    ix = DedupeIndex(8, gated=True)
    ids, new = ix.assign(np.arange(6), 100)
    assert len(new) == 6
    with pytest.raises(DedupeFull):
        ix.assign(np.arange(10, 13), 200)                 # 6 + 3 > 8: nothing admitted
    assert len(ix) == 6 and 10 not in ix
    assert ix.erase([0, 1, 77]) == 2 and 0 not in ix and 1 not in ix and 2 in ix
    ids, new = ix.assign(np.arange(10, 13), 200)
    assert len(new) == 3 and len(ix) == 7


def test_replay_older_than_the_window_is_still_deduplicated():
    """Batch A is never committed (its shard's outage holds the engine's commit); 20 windows
    of other transactions arrive meanwhile; A is replayed after an engine restart: every row
    is a duplicate.  Once the engine commits past A's marks, A's keys may leave."""
    eng = ProcessEngine(standard_dedupe_window=1000, standard_dedupe_capacity=40_000)
    a = np.arange(500, dtype=np.int64) + 10**9
    ids_a = eng.start_standard_array(_batch(a, part=0, mark=700))
    for k in range(40):                                   # 20 windows, committed as they go
        eng.start_standard_array(_batch(np.arange(500) + 2000 * k, part=1, mark=500 * (k + 1)))
        eng.note_committed({1: 500 * (k + 1)})
    assert eng.standard_count == 500 * 41
    before = eng.standard_duplicates
    again = eng.start_standard_array(_batch(a, part=0, mark=800))     # the replay
    np.testing.assert_array_equal(again, ids_a)
    assert eng.standard_duplicates - before == 500 and eng.standard_count == 500 * 41
    st = eng.dedupe_stats()
    assert st["keys"] >= 500 and st["evicted"] > 0
    eng.note_committed({0: 800})                          # A can no longer be re-delivered
    for k in range(3):
        eng.start_standard_array(_batch(np.arange(500) + 10**7 + 1000 * k, part=1, mark=30_000 + k))
        eng.note_committed({1: 30_000 + k})
    assert a[0] not in eng._std_index                     # evicted once committed
    assert eng.dedupe_stats()["keys"] <= 1000 + 500


def test_capacity_refuses_instead_of_evicting_uncommitted():
    eng = ProcessEngine(standard_dedupe_window=100, standard_dedupe_capacity=1000)
    eng.start_standard_array(_batch(np.arange(900), part=3, mark=10))
    with pytest.raises(DedupeFull):
        eng.start_standard_array(_batch(np.arange(900, 1200), part=3, mark=20))
    assert eng.standard_dedupe_full == 1 and eng.standard_count == 900
    eng.note_committed({3: 10})
    eng.start_standard_array(_batch(np.arange(900, 1200), part=3, mark=20))
    assert eng.standard_count == 1200


def test_gates_and_commits_survive_recovery(tmp_path):
    j = str(tmp_path / "kie.jsonl")
    eng = ProcessEngine(journal_path=j, standard_dedupe_window=200, standard_dedupe_capacity=5000)
    old = np.arange(300, dtype=np.int64) + 5_000_000
    ids_old = eng.start_standard_array(_batch(old, part=0, mark=50))
    for k in range(10):
        eng.start_standard_array(_batch(np.arange(300) + 1000 * k, part=1, mark=300 * (k + 1)))
        eng.note_committed({1: 300 * (k + 1)})
    eng.close()
    rec = ProcessEngine.recover(j, standard_dedupe_window=200, standard_dedupe_capacity=5000)
    assert rec.standard_count == 3300
    np.testing.assert_array_equal(rec.start_standard_array(_batch(old, part=0, mark=60)), ids_old)
    assert rec.standard_duplicates == 300 and rec.standard_count == 3300
    assert rec.dedupe_stats()["keys"] <= 200 + 300 + 300     # committed partition-1 keys left
    rec.close()


def test_find_transaction_million_standard_starts_across_shards_and_restart(tmp_path):
    """10^6 standard starts over 4 shards; random transactions are answered by the shard that
    owns them (instance id, route, proba), before and after every shard restarts from its
    journal; a fraud transaction answers its live instance."""
    K, N = 4, 1_000_000
    rng = np.random.default_rng(7)
    tx = rng.permutation(np.arange(N, dtype=np.int64) * 3 + 11)
    proba = rng.random(N).astype(np.float32) * 0.4
    sh = shard_of_tx(tx, K)
    paths = [str(tmp_path / f"kie{k}.jsonl") for k in range(K)]
    engines = [ProcessEngine(journal_path=paths[k], shard=k, shards=K) for k in range(K)]
    ids = np.empty(N, np.int64)
    for lo in range(0, N, 65536):                         # hand-off sized batches
        sl = slice(lo, lo + 65536)
        for k in range(K):
            m = sh[sl] == k
            got = engines[k].start_standard_array(_batch(tx[sl][m], part=k, mark=lo + 65536, proba=proba[sl][m]))
            ids[np.arange(lo, min(N, lo + 65536))[m]] = got
    engines[2].start_fraud({"transaction_id": 99, "customer_id": 1, "amount": 500.0, "proba": 0.97})
    pick = rng.choice(N, 200, replace=False)

    def check(engs):
        for i in pick:
            r = engs[sh[i]].find_transaction(int(tx[i]))
            assert r is not None and r["route"] == "standard"
            assert r["process-instance-id"] == ids[i] and abs(r["proba"] - proba[i]) < 1e-7
            assert engs[(sh[i] + 1) % K].find_transaction(int(tx[i])) is None     # not another shard's
        assert engs[0].find_transaction(10**12) is None
    check(engines)
    for e in engines:
        e.close()
    rec = [ProcessEngine.recover(paths[k], shard=k, shards=K) for k in range(K)]
    check(rec)
    fr = [r.find_transaction(99) for r in rec if r.find_transaction(99)]
    assert len(fr) == 1 and fr[0]["route"] == "fraud" and fr[0]["state"] == "waiting_customer"
    # beyond the in-memory audit: the journal scan still answers
    small = ProcessEngine.recover(paths[sh[pick[0]]], shard=int(sh[pick[0]]), shards=K, standard_audit_rows=1)
    small._std_index = DedupeIndex(8, gated=True)         # forget the in-memory index entirely
    assert small.find_transaction(int(tx[pick[0]])) is None
    deep = small.find_transaction(int(tx[pick[0]]), deep=True)
    assert deep["source"] == "journal" and deep["process-instance-id"] == ids[pick[0]]
    assert abs(deep["proba"] - proba[pick[0]]) < 1e-7
    for r in rec + [small]:
        r.close()


def test_kie_rest_committed_and_by_transaction():
    async def go():
        eng = ProcessEngine(standard_dedupe_window=10, standard_dedupe_capacity=40)
        srv = KieServer(eng, tick_s=0.05)
        c, sp = "ccd-fraud-kjar", "ccd-fraud-kjar.StandardProcess"
        async with TestClient(TestServer(srv.app)) as cl:
            url = f"{BASE}/containers/{c}/processes/{sp}/instances/batch"
            body = encode_columns(_batch(np.arange(30) + 500, part=0, mark=31))
            r = await cl.post(url, data=body, headers={"Content-Type": "application/x-ccfd-columns"})
            assert r.status == 201
            # full of uncommitted keys: 503 (the hand-off retries), not an eviction
            body2 = encode_columns(_batch(np.arange(20) + 900, part=0, mark=52))
            r = await cl.post(url, data=body2, headers={"Content-Type": "application/x-ccfd-columns"})
            assert r.status == 503
            r = await cl.post(f"{BASE}/containers/{c}/processes/{sp}/instances/committed",
                              json={"offsets": {"0": 31}})
            assert r.status == 200
            r = await cl.post(url, data=body2, headers={"Content-Type": "application/x-ccfd-columns"})
            assert r.status == 201
            r = await cl.get(f"{BASE}/containers/{c}/processes/instances/by-transaction/905")
            assert r.status == 200
            got = await r.json()
            assert got["route"] == "standard" and got["process-id"] == "standard" and abs(got["proba"] - 0.01) < 1e-6
            assert (await cl.get(f"{BASE}/containers/{c}/processes/instances/by-transaction/77")).status == 404
            st = await (await cl.get("/rest/stats")).json()
            assert st["standard_dedupe"]["refused_batches"] == 1
    asyncio.new_event_loop().run_until_complete(go())


def test_handoff_delivers_commit_notices_after_starts():
    """The router's hand-off queues a commit notice behind the starts it covers; a run of
    notices is coalesced (max per partition); an in-process sink's DedupeFull is retried."""
    from ccfd_demo_summit_amd.router.handoff import KieHandoff
    eng = ProcessEngine(standard_dedupe_window=10, standard_dedupe_capacity=40)
    h = KieHandoff(eng, workers=1, backoff_s=0.01, max_backoff_s=0.02, max_standard_batch=30)
    h.submit_standard(_batch(np.arange(30), part=0, mark=30))
    h.submit_standard(_batch(np.arange(30, 50), part=0, mark=50))        # needs the notice first
    h.submit_committed({0: 10})
    h.submit_committed({0: 30})
    assert h.drain(0.3) is False                          # held: the second batch does not fit yet
    # FIFO: the notice sits behind the refused batch -- send it on another handle, as the next
    # engine commit would after the earlier batches were acked
    eng.note_committed({0: 30})
    assert h.drain(10.0)
    assert eng.standard_count == 50 and h.retries > 0
    h.close()


def test_journal_header_refuses_another_shard_layout(tmp_path):
    """Instance ids encode (shard, K): a journal written as shard 1 of 4 is refused by a
    process that would decode it as shard 1 of 2."""
    j = str(tmp_path / "kie1.jsonl")
    eng = ProcessEngine(journal_path=j, shard=1, shards=4)
    eng.start_standard_array(_batch(np.arange(10), part=0, mark=10))
    eng.close()
    ok = ProcessEngine.recover(j, shard=1, shards=4)
    assert ok.standard_count == 10
    ok.close()
    with pytest.raises(ValueError, match="shard 1 of 4"):
        ProcessEngine.recover(j, shard=1, shards=2)
