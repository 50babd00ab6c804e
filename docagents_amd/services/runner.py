"""Service entry points: ``python -m docagents_amd.services <name>``.

  gateway | query            HTTP agents (uvicorn) on PORT
  parser  | analysis         queue workers + /healthz server on PORT (errgroup in the reference)
  all                        every agent in one process (in-proc queue unless QUEUE_PROVIDER is set)
  broker                     the native NATS-protocol broker (C++), QUEUE_URL listen address
  kvcache                    the native RESP key-value cache (C++), REDIS_ADDR listen address
  engine                     the MI355X engine server (run under torchrun for multiple GPUs)

Startup sweep: the ``analysis``/``all`` agents re-enqueue parse tasks for documents
stuck in ``processing`` whose chunks never appeared (lost while no worker was connected).
"""
from __future__ import annotations

import asyncio
import os
import signal
import sys

from ..config import load


async def _serve_http(app, port: int, host: str = "0.0.0.0"):
    if os.environ.get("DA_HTTP_SERVER", "native") != "uvicorn":
        from ..api.server import serve
        return await serve(app, host, port)
    import uvicorn
    cfg = uvicorn.Config(app, host=host, port=port, log_level="warning", access_log=False, lifespan="off")
    server = uvicorn.Server(cfg)
    server.install_signal_handlers = lambda: None
    await server.serve()


def _health_app(deps, name):
    from starlette.applications import Starlette
    from starlette.responses import PlainTextResponse
    from starlette.routing import Route

    from ..api.http import Middleware, metrics_response

    async def health(req):
        return PlainTextResponse("ok")

    async def metrics(req):
        return metrics_response()

    return Middleware(Starlette(routes=[Route("/healthz", health), Route("/metrics", metrics)]), deps.log, name)


async def _stop_event():
    stop = asyncio.Event()
    loop = asyncio.get_running_loop()
    for s in (signal.SIGINT, signal.SIGTERM):
        try:
            loop.add_signal_handler(s, stop.set)
        except (NotImplementedError, RuntimeError):
            pass
    return stop


async def run_worker_service(name: str):
    from ..app import build
    from . import analysis, parser
    deps = await build(name)
    _attach_tokenizer(deps)
    stop = await _stop_event()
    deps.log.info(f"{name} worker starting")
    if name == "parser":
        worker = deps.queue.worker("parse", parser.make_handler(deps), stop,
                                   on_permanent_failure=parser.make_failure_hook(deps))
    else:
        await startup_sweep(deps)
        worker = deps.queue.worker("analyze", analysis.make_handler(deps), stop,
                                   on_permanent_failure=analysis.make_failure_hook(deps))
    deps.log.info(f"{name} health endpoint listening", "addr", f":{deps.config.port}")
    http = asyncio.ensure_future(_serve_http(_health_app(deps, name), deps.config.port))
    try:
        await worker  # returns once SIGINT / SIGTERM set ``stop`` and in-flight tasks finished
    finally:
        http.cancel()
        try:
            await http
        except (asyncio.CancelledError, Exception):  # noqa: BLE001
            pass
    deps.log.info(f"{name} worker stopped")


def _attach_tokenizer(deps):
    if deps.config.llm_provider in ("local", "engine", "openai"):
        try:
            from ..models.configs import decoder_config
            from ..models.tokenizer import decoder_tokenizer
            deps.extras["dec_tokenizer"] = decoder_tokenizer(decoder_config(deps.config.llm_arch).vocab)
        except Exception as e:  # noqa: BLE001
            deps.log.warn("decoder tokenizer unavailable; answers will tokenize context on the fly", "err", e)


async def startup_sweep(deps):
    """Re-drive documents stuck in 'processing' (their analyze task was lost), and 'ready' documents
    whose vectors are missing from the engine's shards (e.g. an engine restarted without its
    index directory): both get a fresh analyze task. Only documents older than SWEEP_STUCK_AFTER_S
    count as stuck: a document uploaded while this worker was starting is in flight, not lost
    (the broker redelivers an unacked task itself)."""
    if not hasattr(deps.store, "list_documents") or deps.queue is None:
        return
    import datetime as dt
    import json

    from ..queue.task import TASK_ANALYZE, Task, enqueue_with_retry
    cutoff = dt.datetime.now(dt.timezone.utc) - dt.timedelta(
        seconds=getattr(getattr(deps, "config", None), "sweep_stuck_after_s", 600.0))
    try:
        docs = await deps.store.list_documents("processing")
        for d in docs:
            ca = d.created_at
            if ca is not None and (ca if ca.tzinfo else ca.replace(tzinfo=dt.timezone.utc)) > cutoff:
                continue
            chunks = await deps.store.list_chunks(d.id)
            if chunks:
                body = json.dumps({"document_id": d.id, "chunk_ids": [c.id for c in chunks],
                                   "redrive": True}).encode()
                await enqueue_with_retry(deps.queue, Task(type=TASK_ANALYZE, payload=body), 3, 0.2)
                deps.log.info("re-enqueued stuck document", "document_id", d.id)
        vec = getattr(deps.store, "vectors", None)
        if hasattr(vec, "doc_rows"):
            have = await vec.doc_rows()
            for d in await deps.store.list_documents("ready"):
                chunks = await deps.store.list_chunks(d.id)
                if chunks and have.get(d.id, 0) < len(chunks):
                    body = json.dumps({"document_id": d.id, "chunk_ids": [c.id for c in chunks],
                                       "reindex": True}).encode()
                    await enqueue_with_retry(deps.queue, Task(type=TASK_ANALYZE, payload=body), 3, 0.2)
                    deps.log.info("re-enqueued document with missing vectors", "document_id", d.id,
                                  "indexed", have.get(d.id, 0), "chunks", len(chunks))
    except Exception as e:  # noqa: BLE001
        deps.log.warn("startup sweep failed", "err", e)


async def _loop_lag_monitor(every: float = 0.005):
    """DA_REQ_TIMELINE: record event-loop stalls (a 5 ms sleep that took > 10 ms) as timeline events,
    so a slow hop inside a service can be told apart from a blocked loop."""
    from ..utils import timeline
    loop = asyncio.get_running_loop()
    while True:
        t = loop.time()
        await asyncio.sleep(every)
        lag = loop.time() - t - every
        if lag > 0.005:
            timeline.mark("loop_lag", ms=round(lag * 1000, 2))


async def run_http_service(name: str):
    from ..app import build
    from ..utils import timeline
    deps = await build(name)
    if timeline.enabled():
        asyncio.ensure_future(_loop_lag_monitor())
    # everything built at startup (modules, config, clients) to the permanent generation: full
    # collections under load then scan only what requests allocate
    import gc
    gc.collect()
    gc.freeze()
    if name == "gateway":
        from .gateway import build_app
        deps.log.info("gateway listening", "addr", f":{deps.config.port}")
    else:
        from .query import build_app
        deps.log.info("query service listening", "addr", f":{deps.config.port}")
    await _serve_http(build_app(deps), deps.config.port)


async def run_all():
    """Gateway (PORT) + query (PORT+1) + parser + analysis in one process."""
    from ..app import build
    from ..queue.inproc import InProcBus
    from . import analysis, gateway, parser, query
    cfg = load()
    if "QUEUE_PROVIDER" not in os.environ:
        cfg.queue_provider = "inproc"
    if "CACHE_PROVIDER" not in os.environ:
        cfg.cache_provider = "memory"
    qport = cfg.port + 1
    if "QUERY_SERVICE_URL" not in os.environ:
        cfg.query_service_url = f"http://127.0.0.1:{qport}/api/query"
    deps = await build("all", cfg, bus=InProcBus())
    _attach_tokenizer(deps)
    stop = await _stop_event()
    await startup_sweep(deps)
    deps.log.info("all-in-one listening", "gateway", cfg.port, "query", qport)
    http = [asyncio.ensure_future(_serve_http(gateway.build_app(deps), cfg.port)),
            asyncio.ensure_future(_serve_http(query.build_app(deps), qport))]
    try:
        await asyncio.gather(
            deps.queue.worker("parse", parser.make_handler(deps), stop,
                              on_permanent_failure=parser.make_failure_hook(deps)),
            deps.queue.worker("analyze", analysis.make_handler(deps), stop,
                              on_permanent_failure=analysis.make_failure_hook(deps)),
        )
    finally:
        for t in http:
            t.cancel()
        await asyncio.gather(*http, return_exceptions=True)


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    if not argv:
        print(__doc__)
        return 2
    name = argv[0]
    if name in ("gateway", "query"):
        asyncio.run(run_http_service(name))
    elif name in ("parser", "analysis"):
        asyncio.run(run_worker_service(name))
    elif name == "all":
        asyncio.run(run_all())
    elif name == "broker":
        from ..native import run_broker
        return run_broker(argv[1:])
    elif name == "kvcache":
        from ..native import run_kvserver
        return run_kvserver(argv[1:])
    elif name == "engine":
        from .engine_main import main as engine_main
        return engine_main(argv[1:])
    else:
        print(f"unknown service {name!r}\n{__doc__}", file=sys.stderr)
        return 2
    return 0
