"""Service launcher -- the replacement for the reference's OpenShift objects
(DeploymentConfigs/Services of deploy/*.yaml; README.md:34-537 deployment order).

    python -m ccfd_demo_summit_amd.launch <service> [options]

services:
  kafka-lite   Kafka-protocol broker, --nodes N listeners (dev/CI stand-in for Strimzi); with
               --controller URL --node-id N|auto: one broker process of a replicated cluster
  kafka-controller  membership / leader election / ISR / offsets of a replicated kafka-lite cluster
  seldon       fraud model predict() server            (port 8000, modelfull)
  usertask     user-task model predict() server         (port 5000, ccfd-seldon-model)
  kie          business-process server (KIE REST)       (port 8090)
  notifier     customer notification simulator          (port 8080 health)
  router       compat router: Kafka -> remote Seldon predict() -> KIE   (port 8091)
  engine       GPU streaming engine, one rank per GPU (run under torchrun)  (port 8091+rank)
  producer     transaction producer (synthetic / creditcard.csv)
  demo         everything in one process over an in-process broker
  store        the job's shared KV store (TCPStore) for leases / membership   (port 29400)
  elastic      failure-tolerant scoring rank: partition leases (fail-over, exactly-once
               committed counts) + membership generations whose process group carries the
               global X2 counters; a supervised restart rejoins   (--store, --rank, --world)
  supervise    restart-on-crash supervisor:  supervise [--max-restarts N] -- <cmd...>
  dlq-replay   re-deliver the KIE hand-off dead-letter journal (--dlq PATH) to KIE_SERVER_URL
  operator     FraudDetection CR -> Kubernetes manifests (--render) or a local reconcile
               loop of supervised services (--local); accepts the reference's OpenDataHub CR

Configuration: the reference env var names (BROKER_URL, KAFKA_TOPIC, SELDON_URL, ...),
an optional --config YAML, then flags (ccfd_demo_summit_amd/config.py).
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import sys
import threading
import time

from ..config import load_config


def _broker(cfg, inproc=None, idempotent: bool = False):
    """Kafka client.  ``idempotent``: producers (transactions, notifications, responses) use
    Kafka's idempotent produce, so a batch retried across a broker restart is stored once."""
    if inproc is not None:
        return inproc
    from ..ingest.kafka_wire import KafkaBroker
    return KafkaBroker(cfg.kafka.broker_url, connect_wait_s=120.0,    # wait for the broker to come up
                       idempotent=idempotent)


def _safe(fn, default=None):
    """A consumer poll / commit that survives a broker outage (restart, leader election): the
    error is reported and the caller's loop simply tries again on its next turn."""
    from ..ingest.broker import BrokerError
    try:
        return fn()
    except (BrokerError, OSError, ConnectionError) as e:
        now = time.monotonic()
        if now - _safe.last > 1.0:
            print(f"[launch] broker unavailable: {e!r}"[:300], file=sys.stderr, flush=True)
            _safe.last = now
        time.sleep(0.05)
        return default


_safe.last = 0.0


def _consumer(broker, a, group, topics):
    """Static consumer (every partition), or with --group-membership a Kafka consumer-group
    member whose partitions the coordinator assigns and moves on failure -- how the
    reference's replicated services share a topic (ingest/kafka_group.py)."""
    if getattr(a, "group_membership", False) and hasattr(broker, "group_consumer"):
        return broker.group_consumer(group, topics, session_timeout_s=a.session_timeout)
    return broker.consumer(group, topics)


def _kie_client(cfg, timeout_s: float = 5.0, pool_size: int = 5):
    """The router / engine side of KIE: one KieClient, or a ShardedKieClient over the
    ``kie.shards`` servers KIE_SERVER_URL names (process/sharding.py)."""
    from ..process.sharding import ShardedKieClient
    sk = ShardedKieClient.from_config(cfg.kie, timeout_s=timeout_s, pool_size=pool_size)
    return sk.clients[0] if sk.shards == 1 else sk


def _model(kind: str, weights: str = None, seed: int = 0):
    from ..data import FRAUD_RATE, generate
    from ..models import build_model, load_model
    if weights:
        return load_model(weights)
    X, _ = generate(100_000, seed=seed + 17)
    return build_model(kind, seed=seed, X_ref=X, calibrate_rate=FRAUD_RATE)


def _metrics_app(expose):
    from aiohttp import web

    from ..metrics.exporter import CONTENT_TYPE

    async def handler(_r):
        return web.Response(body=expose(), headers={"Content-Type": CONTENT_TYPE})
    app = web.Application()
    app.router.add_get("/prometheus", handler)
    app.router.add_get("/metrics", handler)
    app.router.add_get("/health/ping", lambda _r: web.json_response({"status": "ok"}))
    return app


def _serve_in_thread(app, host, port):
    """Serve ``app`` on a daemon thread's event loop.  Binds before returning: a port that
    is taken raises OSError here instead of failing silently inside the thread."""
    from aiohttp import web
    ready = threading.Event()
    err = []

    def run():
        loop = asyncio.new_event_loop()
        asyncio.set_event_loop(loop)
        runner = web.AppRunner(app)
        try:
            loop.run_until_complete(runner.setup())
            loop.run_until_complete(web.TCPSite(runner, host, port).start())
        except BaseException as e:          # noqa: BLE001 -- handed to the caller
            err.append(e)
            ready.set()
            return
        ready.set()
        loop.run_forever()
    t = threading.Thread(target=run, daemon=True)
    t.start()
    if not ready.wait(60):
        raise TimeoutError(f"server on {host}:{port} did not start")
    if err:
        raise OSError(f"cannot serve on {host}:{port}: {err[0]!r}") from err[0]
    return t


# ---------------------------------------------------------------------------- services
def cmd_kafka_lite(a, cfg):
    """kafka-lite with every option the operator renders (operator/render.py): durability
    (--data-dir / --fsync), metrics port and retention are forwarded, never dropped."""
    from ..ingest.kafka_lite import main
    argv = ["--host", a.host, "--port", str(a.port or 9092), "--partitions", str(cfg.kafka.partitions),
            "--nodes", str(a.nodes), "--metrics-port", str(a.metrics_port),
            "--retention-batches", str(a.retention_batches), "--fsync", a.fsync]
    if a.advertise:
        argv += ["--advertise", a.advertise]
    if a.data_dir:
        argv += ["--data-dir", a.data_dir]
    if a.controller:                  # one broker process of a replicated cluster
        node = a.node_id
        if node in ("auto", "", None):
            # StatefulSet pod <name>-k is node k + 1
            from ..process.sharding import shard_from_env
            node = str(shard_from_env(None) + 1)
        argv += ["--node-id", str(node), "--controller", a.controller]
    main(argv)


def cmd_kafka_controller(a, cfg):
    """The replicated kafka-lite cluster's controller (ingest/kafka_controller.py)."""
    from ..ingest.kafka_controller import main
    argv = ["--host", a.host, "--port", str(a.port or 9093), "--brokers", str(a.nodes if a.nodes > 1 else 0),
            "--rf", str(a.replication_factor)]
    if a.data_dir:
        argv += ["--data-dir", a.data_dir]
    if a.peers:                       # one member of a replicated controller
        member = a.member_id
        if member in ("auto", "", None):
            # StatefulSet pod <name>-k is member k + 1
            from ..process.sharding import shard_from_env
            member = str(shard_from_env(None) + 1)
        argv += ["--member-id", str(member), "--peers", a.peers]
    main(argv)


def cmd_seldon(a, cfg):
    from ..serving.scorers import make_scorer
    from ..serving.seldon_server import SeldonServer, run
    model = _model(cfg.engine.model, a.weights, cfg.seed)
    scorer = make_scorer(model, cfg.router.fraud_threshold, device=a.device, max_batch=cfg.seldon.max_batch)
    if a.native:
        # C++ epoll front end (csrc/engine/seldon_http.cpp): same routes, JSON and metrics
        from ..serving.native_seldon import NativeSeldonServer
        scorers = [scorer] + [make_scorer(model, cfg.router.fraud_threshold, device=a.device,
                                          max_batch=cfg.seldon.max_batch) for _ in range(a.workers - 1)]
        srv = NativeSeldonServer(scorers if a.workers > 1 else scorer, a.host, a.port or cfg.seldon.port,
                                 cfg.seldon.model_name, cfg.seldon.token, workers=a.workers)
        print(f"[seldon] native {cfg.seldon.model_name} on {getattr(scorer, 'device', 'cpu')} :{srv.port}", flush=True)
        while True:
            time.sleep(3600)
    srv = SeldonServer(scorer, cfg.seldon.model_name, cfg.seldon.token, cfg.seldon.max_batch,
                       cfg.seldon.max_delay_us)
    if a.grpc_port:
        from ..serving.seldon_grpc import SeldonGrpcServer
        gsrv = SeldonGrpcServer(scorer, cfg.seldon.model_name, cfg.seldon.token, cfg.seldon.max_batch,
                                cfg.seldon.max_delay_us, metrics=srv.metrics)

        async def _grpc_up(_app):
            await gsrv.start(a.host, a.grpc_port)

        async def _grpc_down(_app):
            await gsrv.stop()
        srv.app.on_startup.append(_grpc_up)
        srv.app.on_cleanup.append(_grpc_down)
    print(f"[seldon] {cfg.seldon.model_name} on {getattr(scorer, 'device', 'cpu')} :{a.port or cfg.seldon.port}"
          + (f" grpc :{a.grpc_port}" if a.grpc_port else ""), flush=True)
    run(srv, a.host, a.port or cfg.seldon.port)


def cmd_usertask(a, cfg):
    from ..serving.seldon_server import run, usertask_server
    run(usertask_server(cfg.seldon.token), a.host, a.port or 5000)


def cmd_kie(a, cfg):
    from aiohttp import web

    from ..metrics.exporter import KieMetrics
    from ..process.engine import ProcessEngine
    from ..process.kie_server import KieServer
    from ..process.notifier import encode_notification
    from ..process.prediction_service import PredictionService
    from ..serving.client import SeldonClient
    from ..process.sharding import shard_from_env
    shard, shards = shard_from_env(a.shard), max(1, cfg.kie.shards)
    if not 0 <= shard < shards:
        raise SystemExit(f"kie: shard {shard} outside kie.shards={shards}")
    broker = _broker(cfg, idempotent=True)
    topic = cfg.kafka.notification_topic
    # the KIE pod's own SELDON_URL / SELDON_ENDPOINT name ITS prediction-service target (the
    # user-task model, ccd-service.yaml:61-62), not the router's fraud model
    url = os.environ.get("SELDON_URL") or cfg.kie.seldon_url
    endpoint = os.environ.get("SELDON_ENDPOINT") or cfg.kie.seldon_endpoint
    client = SeldonClient(url, endpoint, cfg.seldon.token, cfg.seldon.timeout_ms,
                          cfg.seldon.pool_size) if a.remote_prediction else None
    from ..ingest.producer import BatchingPublisher
    # notifications leave in batches, off the request path; the outbox entry of each (its
    # fraud instance's journal record, written before the start is acknowledged) is cleared
    # once the broker acknowledged it, and re-published after a crash (process/engine.py)
    holder = {}
    pub = BatchingPublisher(broker, topic, on_sent=lambda toks: holder["eng"].mark_notified(toks))
    kw = dict(publish_notification=lambda m: pub.publish(encode_notification(m), token=m["process_id"]),
              kie_metrics=KieMetrics(),
              prediction=PredictionService(cfg.kie.confidence_threshold, client=client), shard=shard, shards=shards,
              standard_dedupe_window=cfg.kie.standard_dedupe_window,
              standard_dedupe_capacity=cfg.kie.standard_dedupe_capacity or None,
              standard_audit_rows=cfg.kie.standard_audit_rows)
    if a.journal and os.path.exists(a.journal):
        # restart after a crash: in-flight instances, timers and the per-transaction dedupe
        # index come back from the journal, so re-sent fraud starts are recognised
        eng = ProcessEngine.recover(a.journal, notification_timeout_s=cfg.kie.notification_timeout_s,
                                    dmn_probability_threshold=cfg.kie.dmn_probability_threshold,
                                    dmn_amount_threshold=cfg.kie.dmn_amount_threshold, **kw)
        print(f"[kie] recovered {len(eng.instances)} instances ({eng.fraud_count} fraud, {eng.standard_count} "
              f"standard) from {a.journal}", flush=True)
    else:
        eng = ProcessEngine.from_config(cfg.kie, journal_path=a.journal, **kw)
    holder["eng"] = eng
    outbox = eng.pending_notifications()
    for m in outbox:                    # notifications whose produce was never acknowledged
        pub.publish(encode_notification(m), token=m["process_id"])
    if outbox:
        print(f"[kie] outbox: re-publishing {len(outbox)} notifications", flush=True)
    srv = KieServer(eng, cfg.kie.container_id, cfg.kie.fraud_process_id, cfg.kie.standard_process_id)
    print(f"[kie] shard {shard} of {shards} on :{a.port or cfg.kie.port}", flush=True)
    from ..ingest.kafka_wire import warm_native
    print(f"[kie] native codecs loaded in {warm_native():.2f} s", flush=True)
    from ..utils.gcpolicy import track_pauses, tune_for_service
    print(f"[kie] gc: {tune_for_service()}", flush=True)
    track_pauses(srv.gc_pauses)
    web.run_app(srv.app, host=a.host, port=a.port or cfg.kie.port, print=None, access_log=None)


def cmd_notifier(a, cfg):
    from aiohttp import web

    from ..ingest.producer import BatchingPublisher
    from ..process.notifier import NotificationService
    broker = _broker(cfg, idempotent=True)
    # replies leave in batches (one produce request per linger period, not per reply); a
    # consumed notification's offset is committed only once its reply is acknowledged
    holder = {}
    pub = BatchingPublisher(broker, cfg.kafka.response_topic, on_sent=lambda toks: holder["ns"].on_published(toks))
    ns = NotificationService(lambda raw, key, tok: pub.publish(raw, token=tok),
                             cfg.notifier.p_reply, cfg.notifier.p_approve, cfg.notifier.mean_delay_s,
                             cfg.notifier.seed, ack_async=True)
    holder["ns"] = ns
    cons = _consumer(broker, a, "notification-service", [cfg.kafka.notification_topic])
    app = web.Application()
    app.router.add_get("/health/ping", lambda _r: web.json_response(dict(status="ok", **ns.stats())))
    _serve_in_thread(app, a.host, a.port or cfg.notifier.port)
    from ..ingest.kafka_wire import warm_native
    warm_native()                       # the reply publisher's codecs, before the first reply
    from ..utils.gcpolicy import tune_for_service
    tune_for_service()
    last_commit = 0.0
    while True:
        for r in _safe(lambda: cons.poll(timeout=0.05, max_records=10_000), []):
            ns.handle(r.value, offset=(r.topic, r.partition, r.offset))
        ns.tick()
        now = time.monotonic()
        if now - last_commit >= 0.05:
            offs = ns.committable()
            own = getattr(cons, "assignment", None)
            if own is not None:
                offs = {tp: o for tp, o in offs.items() if tp in set(own)}
            if offs:
                _safe(lambda: cons.commit(offs))
            last_commit = now


def cmd_router(a, cfg):
    """Reference-topology router: per fetch, POST the batch to the remote Seldon predict()."""
    import numpy as np

    from ..contracts import seldon
    from ..ingest.codec import decode_records
    from ..metrics.exporter import RouterMetrics
    from ..router.router import Router
    from ..router.rules import RuleSet
    from ..serving.client import SeldonClient
    broker = _broker(cfg)
    rm = RouterMetrics()
    kie = _kie_client(cfg)
    router = Router(RuleSet.from_config(cfg.router), kie, rm)
    sc = SeldonClient(cfg.seldon.url, cfg.seldon.endpoint, cfg.seldon.token, cfg.seldon.timeout_ms,
                      cfg.seldon.pool_size)
    _serve_in_thread(_metrics_app(rm.expose), a.host, a.port or cfg.router.port)
    tx = _consumer(broker, a, cfg.kafka.group_id, [cfg.kafka.transactions_topic])
    resp = _consumer(broker, a, cfg.kafka.group_id + "-responses", [cfg.kafka.response_topic])
    notif = _consumer(broker, a, cfg.kafka.group_id + "-notifications", [cfg.kafka.notification_topic])
    while True:
        recs = tx.poll(timeout=0.05, max_records=a.max_batch)
        if recs:
            X, ids, cust = decode_records([r.value for r in recs])
            proba = seldon.proba1_from_response(sc.predict_sync(seldon.build_request(X)))
            router.on_scored(ids, cust, proba, X=X)
            tx.commit()
        for r in resp.poll(max_records=10_000):
            router.on_response(r.value)
        resp.commit()
        for r in notif.poll(max_records=10_000):
            router.on_notification_sent(r.value)
        notif.commit()


def _shard_path(path: str, shard: int) -> str:
    """A per-KIE-shard file next to ``path``: x.rank0.jsonl -> x.rank0.shard2.jsonl."""
    root, ext = os.path.splitext(path)
    return f"{root}.shard{shard}{ext or '.jsonl'}"


def _rank_path(path: str, rank: int) -> str:
    """A per-rank file next to ``path`` (ranks never share a journal): x.jsonl -> x.rank3.jsonl."""
    root, ext = os.path.splitext(path)
    return f"{root}.rank{rank}{ext or '.jsonl'}"


def cmd_engine(a, cfg):
    import numpy as np
    import torch

    from prometheus_client import CollectorRegistry, generate_latest

    from ..metrics.exporter import EngineModelCollector, GpuEngineCollector, MetricsHub
    from ..parallel.dp import broadcast_model, init_distributed, resolve_row_format
    from ..router.handoff import KieHandoff
    from ..router.router import Router
    from ..router.rules import RuleSet
    from ..utils.numa import bind_to_gpu
    from .engine_service import EngineService, EngineServiceConfig, rule_safe_row_format
    ctx = init_distributed()
    bind_to_gpu(ctx.device.index)
    rules = RuleSet.from_config(cfg.router)
    fmt, why = rule_safe_row_format(cfg.engine.model, resolve_row_format(cfg.engine.model, cfg.engine.wire), rules)
    if why:
        print(f"[engine] {why}", flush=True)
    model = _model(cfg.engine.model, a.weights, cfg.seed) if ctx.rank == 0 else None
    dm = broadcast_model(ctx, model, cfg.engine.model, fmt)      # X1 (+ G20 / G32 bin table)
    broker = _broker(cfg)
    hub = MetricsHub()
    kie = _kie_client(cfg, timeout_s=cfg.seldon.timeout_ms / 1e3, pool_size=cfg.seldon.pool_size)
    # fraud starts and response signals go through a bounded async queue with pooled,
    # retried HTTP: a slow or absent KIE never stalls scoring, commits or X2 (router/handoff.py);
    # with a sharded KIE tier one queue (and dead-letter journal) per shard
    from ..router.handoff import DeadLetterQueue, ShardedHandoff
    shards = getattr(kie, "shards", 1)
    dlq_path = _rank_path(cfg.engine.handoff_dlq, ctx.rank) if cfg.engine.handoff_dlq else None
    if shards == 1:
        handoff = KieHandoff(kie, capacity=cfg.engine.handoff_capacity, workers=cfg.engine.handoff_workers,
                             dlq=DeadLetterQueue(dlq_path) if dlq_path else None)
    else:
        dlqs = [DeadLetterQueue(_shard_path(dlq_path, k)) if dlq_path else None for k in range(shards)]
        handoff = ShardedHandoff(kie.clients, dlqs, capacity=cfg.engine.handoff_capacity,
                                 workers=cfg.engine.handoff_workers)
    router = Router(rules, kie, hub.router, standard_mode=cfg.router.standard_mode, handoff=handoff)
    svc = EngineService(ctx, dm, broker, router, EngineServiceConfig(
        topic=cfg.kafka.transactions_topic, group_id=cfg.kafka.group_id, batch=cfg.engine.batch,
        depth=cfg.engine.depth, streams=cfg.engine.streams, input_mode=cfg.engine.input_mode,
        output_mode=cfg.engine.output_mode, exec_mode=cfg.engine.exec_mode,
        flush_us=cfg.engine.max_delay_us, reduce_period_ms=cfg.engine.reduce_period_ms,
        threshold=cfg.router.fraud_threshold, coalesce=cfg.engine.coalesce,
        ingest_threads=cfg.engine.ingest_threads, persist_items=cfg.engine.persist_items,
        standard_mode=cfg.router.standard_mode, scored_capacity=cfg.engine.scored_capacity,
        native_serve=cfg.engine.native_serve,
        model_watch=(a.watch_model or cfg.engine.model_watch or None))).start()
    hub.gpu_registry.register(GpuEngineCollector(svc.metrics_source, rank_label=str(ctx.rank)))
    # the process's node-local rank (torchrun LOCAL_RANK) -- not the device index, which a
    # several-ranks-per-GPU rehearsal (CCFD_DEVICE_MODULO) maps onto the same GPU
    port_rank = int(os.environ.get("LOCAL_RANK", ctx.local_rank))
    # node-local port: every node's (pod's) local rank 0 serves the base port its probes and
    # scrape annotation name, whatever its global rank in a multi-node job
    _serve_in_thread(_metrics_app(lambda: hub.expose_all(include_model=False)), a.host,
                     (a.port or cfg.router.port) + port_rank)
    # the model's own endpoint (the reference's modelfull :8000/prometheus, README.md:292-301):
    # last-request gauges + Seldon engine histograms of THIS rank's streamed traffic
    mport = cfg.seldon.port if a.model_metrics_port is None else a.model_metrics_port
    if mport:
        model_reg = CollectorRegistry()
        model_reg.register(EngineModelCollector(svc.model_source, bins=dm.bins, model_name=cfg.seldon.model_name,
                                                deployment=cfg.seldon.model_name, predictor=cfg.seldon.model_name))
        _serve_in_thread(_metrics_app(lambda: generate_latest(model_reg)), a.host, mport + port_rank)
    print(f"[engine] rank {ctx.rank}: exec_mode {svc.exec_mode}, rows {dm.row_format}, "
          f"model metrics :{(mport + port_rank) if mport else 'off'}", flush=True)
    resp = broker.consumer(cfg.kafka.group_id + "-responses", [cfg.kafka.response_topic]) if ctx.rank == 0 else None
    # the router also watches the notification topic KIE publishes to (router.yaml:57-58)
    notif = (broker.consumer(cfg.kafka.group_id + "-notifications", [cfg.kafka.notification_topic])
             if ctx.rank == 0 else None)
    print(f"[engine] rank {ctx.rank}/{ctx.world} partitions {svc.partitions}", flush=True)
    from ..utils.gcpolicy import tune_for_service
    print(f"[engine] gc: {tune_for_service()}", flush=True)
    # SIGTERM (pod deletion, torchrun shutdown, a supervisor) ends the loop through the
    # `finally` below: the engine drains and its persistent kernel leaves before exit
    import signal

    def _term(*_a):
        raise SystemExit(0)
    signal.signal(signal.SIGTERM, _term)

    def _crash(*_a):
        # SIGUSR1: crash NOW -- no drain, no offset commit, no hand-off flush (what a SIGKILL
        # leaves behind: the rank restarts from its committed offsets), except that a resident
        # persistent kernel is stopped first (a process must never end with one resident)
        try:
            svc.engine.serve_stop()
            svc.engine.emergency_stop(5000)
        finally:
            print(f"[engine] rank {ctx.rank}: crash (SIGUSR1), no commit", flush=True)
            os._exit(137)
    signal.signal(signal.SIGUSR1, _crash)
    resp_wait = None                  # hand-off seq carrying the last polled responses' signals
    try:
        while True:
            svc.step()           # never raises on a KIE outage: the hand-off retries, commits wait
            if resp is not None:
                # customer responses: their offsets are committed only once the signals they
                # became are acknowledged by KIE (like the fraud starts' offsets), so a crash
                # with a KIE outage in flight re-delivers them instead of losing them
                if resp_wait is None or handoff.acked(resp_wait):
                    if resp_wait is not None:
                        if _safe(lambda: resp.commit() or True) is None:
                            continue              # broker outage: commit again next turn
                        resp_wait = None
                    recs = _safe(lambda: resp.poll(max_records=10_000), [])
                    for r in recs:
                        router.on_response(r.value)
                    if recs:
                        resp_wait = router.last_handoff_seq
                for r in _safe(lambda: notif.poll(max_records=10_000), []):
                    router.on_notification_sent(r.value)
                _safe(notif.commit)
    except BaseException as e:
        if not isinstance(e, SystemExit):     # the cause, before the shutdown path runs
            import traceback
            print(f"[engine] rank {ctx.rank} loop failed:", file=sys.stderr, flush=True)
            traceback.print_exc()
            sys.stderr.flush()
        raise
    finally:
        svc.stop()                    # drains; a resident persistent kernel halts here
        handoff.close(drain_s=5.0)
        print(f"[engine] rank {ctx.rank} stopped: rows scored {svc.rows_scored}, hand-off "
              f"{json.dumps(handoff.stats())}", flush=True)


def cmd_producer(a, cfg):
    from ..ingest.producer import ProducerConfig, TransactionProducer
    pc = ProducerConfig.from_env()
    pc.fmt, pc.batch, pc.rate_tx_s, pc.id_base, pc.seed = a.fmt, a.batch, a.rate, a.id_base, a.seed_offset
    if a.csv:
        pc.source, pc.csv_path = "csv", a.csv
    broker = _broker(cfg, idempotent=True)
    broker.stamp_time = True          # ccfd-ts send-time header: the engine's produce -> scored latency
    broker.default_acks = a.acks      # -1: every in-sync replica (replicated kafka-lite)
    broker.max_in_flight = max(1, a.max_in_flight)
    if a.acks == -1:
        broker.RETRIES = 14           # rides out a leader fail-over (~1 s) instead of failing
    prod = TransactionProducer(broker, pc)
    from ..ingest.kafka_wire import warm_native
    warm_native()
    if a.fmt == "txb1" and pc.source == "synthetic":
        prod._txb1_pooled()                 # generate the batch pool before the clock starts
    if a.fmt == "json" and pc.source == "synthetic":
        prod._ensure_pool()                 # render the message pool before the clock starts
        prod._native_json_record_set()      # (and load the native encoder)
        prod._seq = 0
    t0 = time.perf_counter()
    # --seconds with --count 0: a time-bounded open-loop run (deployment benchmarks)
    until = t0 + a.seconds if a.count <= 0 else None
    n = prod.produce(a.count if a.count > 0 else 1 << 62, until=until)
    broker.flush()                    # every pipelined produce answered
    dt = time.perf_counter() - t0
    print(json.dumps({"produced": n, "seconds": round(dt, 3), "tx_s": round(n / max(dt, 1e-9), 1),
                      "topic": pc.topic, "fmt": pc.fmt, "id_base": pc.id_base}), flush=True)


def cmd_demo(a, cfg):
    """All services in one process over an in-process broker; metrics on :8091/prometheus."""
    from ..ingest.broker import InProcBroker
    from ..ingest.producer import ProducerConfig, TransactionProducer
    from ..pipeline import FraudPipeline
    from ..serving.scorers import make_scorer
    model = _model(cfg.engine.model, a.weights, cfg.seed)
    scorer = make_scorer(model, cfg.router.fraud_threshold, device=a.device)
    pipe = FraudPipeline(cfg, scorer, InProcBroker(default_partitions=cfg.kafka.partitions))
    _serve_in_thread(_metrics_app(pipe.metrics.expose_all), a.host, a.port or cfg.router.port)
    prod = TransactionProducer(pipe.broker, ProducerConfig(fmt=a.fmt, batch=a.batch, rate_tx_s=a.rate))
    t_end = time.time() + a.seconds
    while time.time() < t_end:
        prod.produce(a.batch)
        pipe.step()
    pipe.run_until_idle(1000)
    oc = pipe.processes.outcome_counts
    print(json.dumps({"consumed": pipe.stats.consumed, "outcomes": oc,
                      "scorer": getattr(scorer, "device", "cpu")}), flush=True)


def cmd_store(a, cfg):
    """Host the job's TCPStore (it must outlive every rank, so it is its own process)."""
    import datetime

    import torch.distributed as dist
    port = a.port or 29400
    store = dist.TCPStore(a.host if a.host != "0.0.0.0" else "127.0.0.1", port, 1, True,
                          timeout=datetime.timedelta(seconds=3600), wait_for_workers=False)
    print(f"[store] TCPStore on :{port}", flush=True)
    while True:
        time.sleep(3600)
        store.check(["__alive__"])


def cmd_elastic(a, cfg):
    """One failure-tolerant scoring rank (parallel/elastic.py leases + parallel/membership.py)."""
    import datetime

    import numpy as np
    import torch
    import torch.distributed as dist

    from ..metrics.exporter import RouterMetrics
    from ..parallel.elastic import PartitionLeases
    from ..parallel.membership import ElasticCounterReducer, ElasticGroup
    from ..router.router import Router
    from ..router.rules import RuleSet
    from ..serving.scorers import CpuScorer, GpuScorer
    from .elastic_worker import ElasticWorker
    host, _, port = a.store.rpartition(":")
    store = dist.TCPStore(host or "127.0.0.1", int(port), is_master=False,
                          timeout=datetime.timedelta(seconds=120))
    model = _model(cfg.engine.model, a.weights)
    use_gpu = a.device == "gpu" or (a.device == "auto" and torch.cuda.is_available())
    scorer = (GpuScorer(model, cfg.router.fraud_threshold, device_index=a.rank % max(1, torch.cuda.device_count()))
              if use_gpu else CpuScorer(model, cfg.router.fraud_threshold))
    rm = RouterMetrics()
    if a.kie == "local":
        from ..process import ProcessEngine
        sink = ProcessEngine(notification_timeout_s=1e9)
    else:
        sink = _kie_client(cfg)
    router = Router(RuleSet.from_config(cfg.router), sink, rm)
    broker = _broker(cfg)
    leases = PartitionLeases(store, a.rank, a.world, a.partitions, ttl_s=a.ttl)
    worker = ElasticWorker(a.rank, leases, broker, cfg.kafka.transactions_topic, scorer, router,
                           group=cfg.kafka.group_id, max_records=a.max_batch)
    grp = ElasticGroup(store, a.rank, a.world, backend="gloo", ttl_s=a.ttl, timeout_s=max(10.0, 5 * a.ttl))
    x2 = ElasticCounterReducer(grp, 2)
    _serve_in_thread(_metrics_app(rm.expose), a.host, (a.port or cfg.router.port) + a.rank)
    t_end = time.time() + a.seconds if a.seconds > 0 else float("inf")
    last_rows = last_fraud = 0
    while time.time() < t_end and not store.check(["stop"]):
        worker.tick()
        if grp.tick():
            x2.on_regroup()
        rows, fraud = worker.routed
        if rows != last_rows or fraud != last_fraud:
            x2.submit(torch.tensor([rows - last_rows, fraud - last_fraud], dtype=torch.int64))
            last_rows, last_fraud = rows, fraud
        x2.progress()
        t = x2.totals.tolist()
        store.set(f"x2/{a.rank}", f"{grp.gen}|{','.join(map(str, grp.members))}|{t[0]},{t[1]}")
        time.sleep(0.005)
    grp.close()


def cmd_operator(a, cfg):
    """FraudDetection CR (or the reference's OpenDataHub CR) -> Kubernetes manifests
    (--render FILE, '-' = stdout) and/or a local reconcile loop of supervised processes
    (--local; edits of the CR file scale the running deployment)."""
    from ..operator import LocalOperator, dump, load, render, validate
    if not a.cr:
        raise SystemExit("operator: --cr FILE required")
    spec = load(a.cr)
    for n in spec.notes:
        print(f"[operator] note: {n}", file=sys.stderr)
    if a.render:
        manifests = render(spec)
        probs = validate(manifests)
        if probs:
            raise SystemExit("operator: invalid rendering:\n  " + "\n  ".join(probs))
        text = dump(manifests, f"# rendered from {a.cr} by `launch operator --render`\n")
        if a.render == "-":
            sys.stdout.write(text)
        else:
            with open(a.render, "w") as f:
                f.write(text)
    if a.local:
        op = LocalOperator(spec, workdir=os.getcwd(), status_path=a.status)
        t_end = time.time() + a.seconds
        op.run(a.cr, until=(lambda: time.time() >= t_end) if a.seconds > 0 else None)


def cmd_dlq_replay(a, cfg):
    """Re-deliver the hand-off dead-letter journal (router/handoff.py DeadLetterQueue) to
    KIE_SERVER_URL: every pending entry exactly once; prints a JSON summary."""
    from ..router.handoff import DeadLetterQueue
    path = a.dlq or cfg.engine.handoff_dlq
    if not path:
        raise SystemExit("dlq-replay: --dlq PATH (or CCFD_HANDOFF_DLQ) is required")
    kie = _kie_client(cfg, timeout_s=cfg.seldon.timeout_ms / 1e3)     # routes a sharded tier's entries
    q = DeadLetterQueue(path)
    res = q.replay(kie)
    q.close()
    print(json.dumps(dict(res, dlq=path)), flush=True)
    if res["failed"]:
        sys.exit(1)


def cmd_supervise(a, cfg):
    from .supervisor import supervise
    sys.exit(supervise(a.cmd, max_restarts=a.max_restarts, backoff_s=a.backoff))


def parse_args(argv=None) -> argparse.Namespace:
    """Service name, options (before or after it), and for ``supervise`` the child command
    after ``--``."""
    argv = list(sys.argv[1:] if argv is None else argv)
    cmd = []
    if "--" in argv:
        i = argv.index("--")
        argv, cmd = argv[:i], argv[i + 1:]
    ap = argparse.ArgumentParser(prog="python -m ccfd_demo_summit_amd.launch", description=__doc__,
                                 formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("service", choices=["kafka-lite", "kafka-controller", "seldon", "usertask", "kie", "notifier", "router",
                                        "engine", "producer", "demo", "store", "elastic", "supervise",
                                        "operator", "dlq-replay"])
    ap.add_argument("--config", default=None)
    ap.add_argument("--nodes", type=int, default=1, help="kafka-lite: broker listeners (port, port+1, ...)")
    ap.add_argument("--replication-factor", type=int, default=3,
                    help="kafka-controller: copies of every partition of a new topic")
    ap.add_argument("--advertise", default=None, help="kafka-lite: broker host name clients are given")
    ap.add_argument("--data-dir", default=None,
                    help="kafka-lite: durable log + committed-offset directory (restart recovers from it)")
    ap.add_argument("--fsync", default="interval", choices=["always", "interval", "never"],
                    help="kafka-lite: durability flush policy of --data-dir")
    ap.add_argument("--metrics-port", type=int, default=9404, help="kafka-lite: Prometheus /metrics (0 = off)")
    ap.add_argument("--retention-batches", type=int, default=0,
                    help="kafka-lite: record batches kept per partition (0 = the broker default)")
    ap.add_argument("--node-id", default=None,
                    help="kafka-lite replicated: this broker's node id, or 'auto' (pod ordinal + 1)")
    ap.add_argument("--controller", default=None,
                    help="kafka-lite replicated: the controller's URL, or its members' URLs comma-separated")
    ap.add_argument("--member-id", default=None,
                    help="kafka-controller replicated: this member's id in --peers, or 'auto' (pod ordinal + 1)")
    ap.add_argument("--peers", default=None,
                    help="kafka-controller replicated: every member as id=url, comma-separated")
    ap.add_argument("--cr", default=None, help="operator: FraudDetection (or OpenDataHub) CR file")
    ap.add_argument("--render", default=None, help="operator: write Kubernetes manifests here ('-' = stdout)")
    ap.add_argument("--local", action="store_true", help="operator: reconcile the CR into local processes")
    ap.add_argument("--status", default=None, help="operator --local: status JSON file")
    ap.add_argument("--rules", default=None, help="router/engine/demo: routing rule file (overrides ROUTER_RULES)")
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=None)
    ap.add_argument("--watch-model", default=None, help="engine: hot-swap weights when this file changes")
    ap.add_argument("--model-metrics-port", type=int, default=None,
                    help="engine: port (+ local rank) of the model's /prometheus (proba_1 / Amount / V17 / V10, "
                         "seldon_api_engine_*); default SELDON port 8000, 0 = off")
    ap.add_argument("--grpc-port", type=int, default=0, help="seldon: also serve seldon.protos gRPC Predict")
    ap.add_argument("--native", action="store_true", help="seldon: C++ epoll REST front end (dynamic GPU batching)")
    ap.add_argument("--workers", type=int, default=1, help="seldon --native: epoll worker threads (one engine each)")
    ap.add_argument("--weights", default=None, help="safetensors model file (models.save_model)")
    ap.add_argument("--device", default="auto", choices=["auto", "gpu", "cpu"])
    ap.add_argument("--journal", default=None, help="KIE: append-only process journal for recovery")
    ap.add_argument("--shard", type=int, default=-1,
                    help="KIE: this server's shard of kie.shards (-1 = CCFD_KIE_SHARD or the pod ordinal)")
    ap.add_argument("--dlq", default=None, help="dlq-replay: the hand-off dead-letter journal to re-deliver")
    ap.add_argument("--remote-prediction", action="store_true", help="KIE: call the user-task model over HTTP")
    ap.add_argument("--fmt", default="json", choices=["json", "txb1"])
    ap.add_argument("--acks", type=int, default=1, choices=[0, 1, -1],
                    help="producer: 1 = the leader, -1 = every in-sync replica (acks=all)")
    ap.add_argument("--max-in-flight", type=int, default=1,
                    help="producer: produce requests in flight per producer (pipelined; idempotent order kept)")
    ap.add_argument("--batch", type=int, default=None,
                    help="producer: JSON messages per produce request (default 1024) / TXB1 rows per "
                         "message (default 4096); 1024-message requests keep the RF-3 produce -> scored "
                         "p99 at ~4 ms (4096: ~7-13 ms, docs/ROUND6.md section 5)")
    ap.add_argument("--rate", type=float, default=0.0)
    ap.add_argument("--count", type=int, default=100_000, help="producer: transactions (0 = run --seconds)")
    ap.add_argument("--id-base", type=int, default=0, help="producer: first transaction id")
    ap.add_argument("--seed-offset", type=int, default=0, help="producer: synthetic data seed")
    ap.add_argument("--csv", default=None)
    ap.add_argument("--seconds", type=float, default=10.0)
    ap.add_argument("--max-batch", type=int, default=4096)
    ap.add_argument("--max-restarts", type=int, default=10)
    ap.add_argument("--backoff", type=float, default=1.0)
    ap.add_argument("--group-membership", action="store_true",
                    help="router/notifier: join the Kafka consumer group (coordinator-assigned partitions)")
    ap.add_argument("--session-timeout", type=float, default=10.0, help="consumer-group session timeout (s)")
    ap.add_argument("--store", default="127.0.0.1:29400", help="elastic: host:port of the job's TCPStore")
    ap.add_argument("--rank", type=int, default=int(os.environ.get("RANK", "0")))
    ap.add_argument("--world", type=int, default=int(os.environ.get("WORLD_SIZE", "1")))
    ap.add_argument("--partitions", type=int, default=0, help="elastic: topic partitions (0 = 2 x world)")
    ap.add_argument("--ttl", type=float, default=2.0, help="elastic: lease / heartbeat ttl (s)")
    ap.add_argument("--kie", default="remote", choices=["remote", "local"],
                    help="elastic: fraud hand-off to KIE_SERVER_URL or an in-process engine")
    a = ap.parse_args(argv)
    a.cmd = cmd
    if a.batch is None:
        a.batch = 1024 if a.fmt == "json" else 4096
    if a.service == "elastic" and a.partitions <= 0:
        a.partitions = 2 * a.world
    if a.service in ("elastic", "operator") and a.seconds == 10.0 and "--seconds" not in argv:
        a.seconds = 0.0                 # elastic ranks / the operator run until stopped
    return a


def main(argv=None):
    a = parse_args(argv)
    cfg = load_config(a.config, overrides={"router.rules": a.rules} if a.rules else None)
    globals()["cmd_" + a.service.replace("-", "_")](a, cfg)


if __name__ == "__main__":
    main()
