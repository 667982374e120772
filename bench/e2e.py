"""End-to-end streaming benchmark: Kafka ingest -> GPU scoring ->
router -> fraud business process -> customer notification -> response -> process signal,
with the Prometheus counters checked against the scored volume.

Per rank (one per MI355X under torchrun, partitions p % W == rank):

  producer thread --TXB1 4096-row batches--> broker (in-process, or kafka-lite speaking the
  Kafka wire protocol over 127.0.0.1) --> EngineService (ingest thread -> pinned ring ->
  coalesced fused-kernel launches -> flagged rows) --> Router --> ProcessEngine (in-process
  KIE: fraud BP, notification publish, timers, DMN) --> notification service --> response
  topic --> Router.on_response --> process signal.

The producer runs open-loop at ``--rate`` tx/s per rank (0 = as fast as the pipeline
absorbs, with back-pressure on consumer lag so retention never drops unconsumed data).
Reported: sustained scored tx/s (whole job), ring-arrival -> scored latency p50/p99,
fraud processes started, notifications/responses, and whether the Prometheus
``transaction_incoming_total`` equals the rows scored.

    python bench/e2e.py --seconds 20 --broker kafka-lite
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 bench/e2e.py --seconds 20 --allow-isolated

Topology: every rank builds its OWN broker, producer, KIE and notifier in-process, so at
N > 1 this measures N isolated stacks, not one topic sharded over N GPUs with one KIE
(config 5 as deployed).  The JSON line says so (``topology``); an N > 1 run is refused
unless ``--allow-isolated``.  The deployed topology -- separate processes, one shared
kafka-lite topic, torchrun engine ranks, one KIE -- is bench/deploy_topology.py.
"""
from __future__ import annotations

import argparse
import json
import sys
import threading
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def _prom(hub) -> dict:
    text = hub.router.expose().decode() if hasattr(hub.router, "expose") else ""
    prom = {}
    for line in text.splitlines():
        for name in ("transaction_incoming_total", "notifications_outgoing_total"):
            if line.startswith(name + " "):
                prom[name] = float(line.split()[-1])
    return prom


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=20.0)
    ap.add_argument("--warmup", type=float, default=3.0)
    ap.add_argument("--broker", default="inproc", choices=["inproc", "kafka-lite"])
    ap.add_argument("--rate", type=float, default=0.0, help="tx/s per rank (0 = max)")
    ap.add_argument("--batch", type=int, default=4096, help="rows per TXB1 message / micro-batch")
    ap.add_argument("--partitions-per-rank", type=int, default=4)
    ap.add_argument("--max-lag-msgs", type=int, default=64, help="producer back-pressure (messages)")
    ap.add_argument("--model", default="mlp", choices=["mlp", "lr", "gbdt"],
                    help="gbdt: 100x6 oblivious ensemble on G32 rows (binned at ingest)")
    ap.add_argument("--flush-us", type=int, default=500, help="deadline flush of partial micro-batches")
    ap.add_argument("--fmt", default="txb1", choices=["txb1", "json"],
                    help="txb1: one columnar batch per message; json: one transaction per message")
    ap.add_argument("--python-ingest", action="store_true", help="kafka-lite: use the Python consumer thread")
    ap.add_argument("--prefill-s", type=float, default=0.0,
                    help="consumer-only mode: the producer fills the topic for this long BEFORE the "
                         "engine starts and stops there; the timed window then measures ingest + "
                         "scoring capacity alone (engine vs producer/broker capacity)")
    ap.add_argument("--kafka-nodes", type=int, default=1, help="kafka-lite broker listeners")
    ap.add_argument("--ingest-threads", type=int, default=0,
                    help="native consumer threads per rank (0 = 1 for TXB1, one per partition for JSON)")
    ap.add_argument("--allow-isolated", action="store_true",
                    help="run at N > 1 ranks anyway: N private broker/KIE stacks (labelled topology "
                         "isolated-per-rank); the shared deployed topology is bench/deploy_topology.py")
    ap.add_argument("--out", default=None)
    args = ap.parse_args(argv)
    import os as _os
    if int(_os.environ.get("WORLD_SIZE", "1")) > 1 and not args.allow_isolated:
        raise SystemExit("bench/e2e.py at WORLD_SIZE > 1 builds one private broker + KIE per rank (isolated "
                         "stacks, not config 5): use bench/deploy_topology.py --ranks N for the shared "
                         "topology, or pass --allow-isolated to label the run as such")

    import torch
    from ccfd_demo_summit_amd.config import load_config
    from ccfd_demo_summit_amd.contracts import TxBatch
    from ccfd_demo_summit_amd.data import FRAUD_RATE, generate
    from ccfd_demo_summit_amd.ingest.broker import InProcBroker
    from ccfd_demo_summit_amd.launch.engine_service import EngineService, EngineServiceConfig
    from ccfd_demo_summit_amd.metrics.exporter import MetricsHub
    from ccfd_demo_summit_amd.models import build_model
    from ccfd_demo_summit_amd.ops.kernels import DeviceModel
    from ccfd_demo_summit_amd.parallel import all_max, all_sum, barrier, hist_quantile, init_distributed
    from ccfd_demo_summit_amd.process import NotificationService, PredictionService, ProcessEngine
    from ccfd_demo_summit_amd.process.notifier import encode_notification
    from ccfd_demo_summit_amd.router.router import Router
    from ccfd_demo_summit_amd.router.rules import RuleSet

    ctx = init_distributed()
    dev = ctx.device
    cfg = load_config(None)
    k = cfg.kafka
    P = args.partitions_per_rank
    lag_limit = args.max_lag_msgs * (args.batch if args.fmt == "json" else 1)   # in messages
    prefill = args.prefill_s > 0
    # notification / response topics stay in-process (side channels of this rank); the
    # transactions topic is the in-process broker or kafka-lite's verbatim batch store
    store = InProcBroker(default_partitions=P, retention=None if prefill else 4 * lag_limit)
    tx_store = store
    server = None
    if args.broker == "kafka-lite":
        from ccfd_demo_summit_amd.ingest.kafka_lite import KafkaLiteCluster
        from ccfd_demo_summit_amd.ingest.kafka_wire import KafkaBroker
        server = KafkaLiteCluster(args.kafka_nodes, "127.0.0.1", 0, default_partitions=P,
                                  retention_batches=None if prefill else 4 * args.max_lag_msgs).start_in_thread()
        tx_store = server.store
        broker = KafkaBroker(server.bootstrap_all)
        prod_broker = KafkaBroker(server.bootstrap_all)
    else:
        broker = prod_broker = store
    for t in (k.notification_topic, k.response_topic):
        store.create_topic(t, P)
    tx_store.create_topic(k.transactions_topic, P)

    # model (same random-init + calibration as bench.py), W64 rows (G32 for the GBDT)
    Xcal, _ = generate(200_000, seed=999)
    model = build_model(args.model, seed=0, X_ref=Xcal, calibrate_rate=FRAUD_RATE)
    bins = None
    if args.model == "gbdt":                  # G20 rows when the bin table fits 5 bits, else G32
        spec = model.bin_spec()
        bins = spec.with_bits(5) if spec.fits_g20 else spec
    dm = DeviceModel(model, dev, wire=args.model != "gbdt", bins=bins)

    hub = MetricsHub()
    processes = ProcessEngine(cfg.kie.notification_timeout_s, cfg.kie.dmn_probability_threshold,
                              cfg.kie.dmn_amount_threshold, kie_metrics=hub.kie,
                              prediction=PredictionService(cfg.kie.confidence_threshold),
                              publish_notification=lambda msg: (store.produce(
                                  k.notification_topic, encode_notification(msg), key=str(msg.get("customer_id")).encode()),
                                  router.on_notification_sent(msg)))
    router = Router(RuleSet.threshold(cfg.router.fraud_threshold), processes, hub.router)
    notifier = NotificationService(lambda raw, key: store.produce(k.response_topic, raw, key=key),
                                   cfg.notifier.p_reply, cfg.notifier.p_approve, 0.05, 7)
    svc = EngineService(ctx, dm, broker, router, EngineServiceConfig(
        topic=k.transactions_topic, group_id=k.group_id, batch=args.batch, depth=32, streams=4,
        ring_rows=1 << 20, flush_us=args.flush_us, run_budget_us=2000, reduce_period_ms=10.0,
        threshold=cfg.router.fraud_threshold, coalesce=8, max_fetch=64,
        native_ingest=not args.python_ingest,
        # JSON parsing and G20 / G32 binning (GBDT) are per-row work on the ingest thread: one
        # consumer thread per partition; TXB1 into W64 / f32 rows is a copy, one thread suffices
        ingest_threads=args.ingest_threads or (P if args.fmt == "json" or dm.row_format in ("g20", "g32") else 1)),
        partitions=list(range(P)))
    notif_c = store.consumer("notification-service", [k.notification_topic])
    resp_c = store.consumer(k.group_id + "-responses", [k.response_topic])

    # producer: pre-encoded TXB1 messages, ids patched per message (unique transaction ids)
    pool = []
    for i in range(8):
        X, _ = generate(args.batch, seed=1000 * ctx.rank + i)
        b = TxBatch(ids=np.zeros(args.batch, np.uint64),
                    customer=np.random.default_rng(i).integers(0, 1_000_000, args.batch, dtype=np.uint32),
                    features=X)
        pool.append(bytearray(b.encode()))
    stop = threading.Event()
    produced = [0]
    id_base = np.uint64(ctx.rank) << np.uint64(48)
    if args.fmt == "json":                  # per-message JSON: pre-rendered tails, ids formatted per batch
        from ccfd_demo_summit_amd.contracts import FEATURE_NAMES
        Xj, _ = generate(args.batch, seed=77 + ctx.rank)
        tails = [(",\"customer_id\":%d," % (i % 100_000) + ",".join(
            f'"{n}":{float(v):.6g}' for n, v in zip(FEATURE_NAMES, Xj[i])) + "}").encode() for i in range(args.batch)]

    def producer(until=None):
        seq = producer.seq
        t0 = time.perf_counter()
        while not stop.is_set() and (until is None or time.perf_counter() < until):
            if args.rate > 0 and produced[0] > args.rate * (time.perf_counter() - t0):
                time.sleep(0.0002)
                continue
            if until is None and tx_store.lag(k.group_id, k.transactions_topic) > lag_limit:
                time.sleep(0.0002)
                continue
            if args.fmt == "json":
                b0 = int(id_base) + seq * args.batch
                msgs = [b'{"id":%d' % (b0 + i) + t for i, t in enumerate(tails)]
                prod_broker.produce_many(k.transactions_topic, msgs, partition=seq % P)
            else:
                msg = pool[seq % len(pool)]
                ids = np.frombuffer(msg, np.uint64, args.batch, 32)
                ids[:] = id_base + np.uint64(seq * args.batch) + np.arange(args.batch, dtype=np.uint64)
                prod_broker.produce(k.transactions_topic, bytes(msg), partition=seq % P)
            produced[0] += args.batch
            seq += 1
        producer.seq = seq
    producer.seq = 0

    th = threading.Thread(target=producer, daemon=True, name="producer")
    if prefill:                                     # fill the topic first, untimed
        tp = time.perf_counter()
        producer(until=tp + args.prefill_s)
        prefill_rate = produced[0] / (time.perf_counter() - tp)
    svc.start()
    if not prefill:
        th.start()

    def loop_until(t_end):
        while time.perf_counter() < t_end:
            svc.step()
            for r in notif_c.poll(max_records=10_000):
                notifier.handle(r.value)
            notif_c.commit()
            notifier.tick()
            for r in resp_c.poll(max_records=10_000):
                router.on_response(r.value)
            resp_c.commit()
            processes.tick()

    loop_until(time.perf_counter() + args.warmup)
    svc.reset_stats()
    rows0 = svc.rows_scored
    fr0 = router.fraud_started
    sig0 = router.signals_ok
    notif0 = _prom(hub).get("notifications_outgoing_total", 0.0)
    inc0 = _prom(hub).get("transaction_incoming_total", 0.0)
    def kc_totals():
        tot = {}
        for kc in svc.natives or []:
            for k, v in kc.stats().items():
                tot[k] = tot.get(k, 0) + v
        return tot
    kc0 = kc_totals()
    barrier(ctx)
    t0 = time.perf_counter()
    loop_until(t0 + args.seconds)
    elapsed = time.perf_counter() - t0
    kc1 = kc_totals()
    rows = svc.rows_scored - rows0
    stop.set()
    if th.is_alive():
        th.join(5)
    svc.flush_epochs()                              # collective: paired X2 reductions on every rank
    lat = svc.latency_hist()                        # cumulative since reset
    tot = all_sum(ctx, float(rows))
    el = all_max(ctx, elapsed)
    prom = _prom(hub)
    incoming = prom.get("transaction_incoming_total")
    out = {
        "metric": "end-to-end tx/s (Kafka ingest -> GPU score -> route -> BP -> notify)",
        # in-process services; at N > 1 one private stack per rank (see the module doc)
        "topology": "single-process" if ctx.world == 1 else "isolated-per-rank",
        "value": round(tot / el, 1), "unit": "tx/s", "n_gpus": ctx.world, "seconds": round(el, 2),
        "broker": args.broker, "rate_per_rank": args.rate, "micro_batch": args.batch, "model": args.model, "row_format": dm.row_format,
        "flush_us": args.flush_us, "fmt": args.fmt,
        "ingest": "python" if (args.python_ingest or args.broker == "inproc") else "native",
        "ring_arrival_to_scored_p50_us": round(hist_quantile(lat, 0.5) / 1e3, 1),
        "ring_arrival_to_scored_p99_us": round(hist_quantile(lat, 0.99) / 1e3, 1),
        # every counter below is a delta over the timed window (rank 0)
        "fraud_processes_started_rank0": router.fraud_started - fr0,
        "notifications_rank0": prom.get("notifications_outgoing_total", 0.0) - notif0,
        "responses_signalled_rank0": router.signals_ok - sig0,
        "prometheus_transaction_incoming_rank0": (incoming or 0.0) - inc0,
        "rows_scored_rank0": svc.rows_scored - rows0,
        "prometheus_transaction_incoming_total_rank0": incoming,
        "rows_scored_rank0_total": svc.rows_scored,
        "producer_lag_msgs_rank0": tx_store.lag(k.group_id, k.transactions_topic),
        "mode": "consumer-only (pre-filled topic)" if prefill else "producer running",
        "prefill_producer_tx_s_rank0": round(prefill_rate, 1) if prefill else None,
        "kafka_nodes": args.kafka_nodes if args.broker == "kafka-lite" else None,
        "ingest_threads": len(svc.natives) if svc.natives else None,
    }
    if kc1:
        # where the native consumer threads spent the window (rank 0): waiting on the broker,
        # parsing responses, writing / encoding rows into the rings, blocked on full rings
        d = {k: kc1.get(k, 0) - kc0.get(k, 0) for k in kc1}
        th = max(1, len(svc.natives)) * elapsed
        rows_in = max(1, d.get("rows", 0))
        out["ingest_attribution_rank0"] = {
            "thread_seconds": round(th, 2),
            "broker_io_frac": round(d["io_ns"] * 1e-9 / th, 3),
            "parse_frac": round((d["handle_ns"] - d["encode_ns"] - d["ring_wait_ns"]) * 1e-9 / th, 3),
            "encode_frac": round(d["encode_ns"] * 1e-9 / th, 3),
            "ring_full_wait_frac": round(d["ring_wait_ns"] * 1e-9 / th, 3),
            "encode_ns_per_row": round(d["encode_ns"] / rows_in, 2),
            "rows_ingested": d.get("rows", 0)}
    if ctx.rank == 0:
        print(json.dumps(out), flush=True)
        if args.out:
            Path(args.out).write_text(json.dumps(out) + "\n")
    svc.stop()
    if server is not None:
        server.stop()
    if ctx.initialized:
        import torch.distributed as dist
        barrier(ctx)
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
