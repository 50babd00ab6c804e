"""Composition root: build each agent's dependency bundle from the config
(internal/app/deps.go:19-267).

Providers (all reference keys accepted; the reference's single valid option each — postgres, nats,
openai, redis — map onto the in-repo MI355X-native equivalents):

  STORE_PROVIDER   sqlite (default; "postgres" -> sqlite metadata)      VECTOR_PROVIDER sqlite|engine|local
  QUEUE_PROVIDER   broker (= nats wire protocol) | nats | inproc
  LLM_PROVIDER     local | engine | stub ("openai" -> engine)           EMBEDDER_PROVIDER (default: LLM_PROVIDER)
  CACHE_PROVIDER   kv (= redis wire protocol) | redis | memory | noop    (kv failure -> noop, deps.go:129-134)
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field

from .cache.cache import KVCache, MemoryCache, NoOpCache
from .config import Config, load
from .providers import LocalEmbedder, LocalLLM, RemoteEmbedder, RemoteLLM, StubEmbedder, StubLLM
from .store.sqlite_store import CompositeStore, SqliteMeta
from .utils.log import Logger, new as new_logger


@dataclass
class Deps:
    config: Config
    log: Logger
    store: object = None
    queue: object = None
    llm: object = None
    embedder: object = None
    cache: object = None
    engine_client: object = None
    extras: dict = field(default_factory=dict)


_ENGINES = {}


def local_engine(cfg: Config):
    """One in-process Engine per config (LLM_PROVIDER=local)."""
    key = (cfg.embed_arch, cfg.llm_arch)
    if key not in _ENGINES:
        import torch
        from .engine.engine import Engine
        dev = "cuda" if torch.cuda.is_available() else "cpu"
        _ENGINES[key] = Engine(cfg.embed_arch, cfg.llm_arch, dev, seed=cfg.seed, max_batch=cfg.max_batch,
                               kv_cache_gb=cfg.kv_cache_gb, temperature=cfg.temperature, max_new_tokens=cfg.max_new_tokens,
                               summary_max_new=cfg.summary_max_new_tokens, index_kind=cfg.index_kind,
                               ivf_lists=cfg.ivf_lists, ivf_probes=cfg.ivf_probes,
                               enc_dtype="fp8" if cfg.dtype == "fp8" else "bf16",
                               max_seq=4096 if dev == "cuda" else 1024)
    return _ENGINES[key]


async def engine_client(cfg: Config, deps: Deps):
    if deps.engine_client is None:
        from .engine.rpc import EngineCluster
        url = cfg.engine_url or "tcp://127.0.0.1:9090"
        deps.engine_client = await EngineCluster(url).connect(retries=40, delay=0.25)
    return deps.engine_client


def _vector_provider(cfg: Config) -> str:
    v = os.environ.get("VECTOR_PROVIDER", "")
    if v:
        return v
    p = cfg.effective_embedder_provider()
    return {"engine": "engine", "openai": "engine", "local": "local"}.get(p, "sqlite")


async def build_store(cfg: Config, log: Logger, deps: Deps):
    if cfg.store_provider not in ("sqlite", "postgres", "memory"):
        raise ValueError(f"invalid STORE_PROVIDER: {cfg.store_provider} (valid options: sqlite, postgres, memory)")
    path = ":memory:" if cfg.store_provider == "memory" else cfg.sqlite_path()
    meta = SqliteMeta(path)
    vp = _vector_provider(cfg)
    if vp == "engine":
        from .store.vectors import EngineVectors
        vectors = EngineVectors(await engine_client(cfg, deps))
    elif vp == "local":
        from .store.vectors import LocalVectors
        vectors = LocalVectors(local_engine(cfg).index)
    else:
        from .store.sqlite_vectors import SqliteVectors
        vectors = SqliteVectors(meta)
    log.info("using store", "metadata", path, "vectors", vp)
    direct = vp == "engine" and cfg.effective_embedder_provider() in ("engine", "openai")
    return CompositeStore(meta, vectors, min_similarity=cfg.min_similarity, direct_embed=direct)


def worker_concurrency(cfg: Config) -> int:
    """Tasks one worker runs at once. The reference handles one message at a time per replica
    (internal/queue/nats.go:43-45); with the GPU engine behind the agents, concurrent tasks are
    what lets the engine batch summaries/embeddings across documents, so the default is 32 there."""
    if cfg.worker_concurrency > 0:
        return cfg.worker_concurrency
    return 32 if cfg.llm_provider in ("engine", "openai", "local") else 1


async def build_queue(cfg: Config, log: Logger, bus=None):
    p = cfg.queue_provider
    if p == "inproc":
        from .queue.inproc import InProcBus, InProcQueue
        return InProcQueue(bus or InProcBus(), log, concurrency=worker_concurrency(cfg))
    if p in ("broker", "nats"):
        if not cfg.queue_url:
            raise ValueError(f"QUEUE_URL is required when QUEUE_PROVIDER={p}")
        from .queue.broker_client import BrokerQueue
        q = BrokerQueue(cfg.queue_url, log, concurrency=worker_concurrency(cfg))
        await q.connect()
        log.info("using broker queue", "url", cfg.queue_url)
        return q
    raise ValueError(f"invalid QUEUE_PROVIDER: {p} (valid options: broker, nats, inproc)")


async def build_llm(cfg: Config, log: Logger, deps: Deps):
    p = cfg.llm_provider
    if p == "stub":
        return StubLLM()
    if p == "local":
        return LocalLLM(local_engine(cfg))
    if p in ("engine", "openai"):
        return RemoteLLM(await engine_client(cfg, deps))
    raise ValueError(f"invalid LLM_PROVIDER: {p} (valid options: local, engine, stub)")


async def build_embedder(cfg: Config, log: Logger, deps: Deps):
    p = cfg.effective_embedder_provider()
    if p == "stub":
        return StubEmbedder(cfg.embed_dim or 768)
    if p == "local":
        return LocalEmbedder(local_engine(cfg))
    if p in ("engine", "openai"):
        return RemoteEmbedder(await engine_client(cfg, deps))
    raise ValueError(f"invalid embedder provider: {p} (valid options: local, engine, stub)")


async def build_cache(cfg: Config, log: Logger):
    p = cfg.cache_provider
    if p == "noop":
        return NoOpCache()
    if p == "memory":
        return MemoryCache()
    if p in ("kv", "redis"):
        try:
            c = await KVCache(cfg.redis_addr, cfg.redis_password).connect()
            log.info("using kv cache", "addr", cfg.redis_addr, "ttl_seconds", cfg.cache_ttl)
            return c
        except Exception as e:  # noqa: BLE001 - cache is optional (deps.go:129-134)
            log.warn("failed to initialize cache, continuing without caching", "err", e)
            return NoOpCache()
    raise ValueError(f"invalid CACHE_PROVIDER: {p} (valid options: kv, redis, memory, noop)")


async def build(service: str, cfg: Config | None = None, bus=None) -> Deps:
    cfg = cfg or load()
    log = new_logger(cfg.log_level)
    deps = Deps(cfg, log)
    deps.store = await build_store(cfg, log, deps)
    if service in ("gateway", "parser", "analysis", "all"):
        deps.queue = await build_queue(cfg, log, bus)
    if service in ("analysis", "query", "all"):
        deps.llm = await build_llm(cfg, log, deps)
        deps.embedder = await build_embedder(cfg, log, deps)
    if service in ("query", "all"):
        deps.cache = await build_cache(cfg, log)
    return deps
