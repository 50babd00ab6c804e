"""Environment configuration.

Accepts every key of the reference (internal/config/config.go:11-42) with the same defaults, plus
the keys of the MI355X engine. Like the reference's ``Load`` (config.go:45-51), a
value that fails to parse is logged and the default is kept.
"""
from __future__ import annotations

import dataclasses
import logging
import os
from dataclasses import dataclass, field, fields

_log = logging.getLogger("docagents.config")


def _env(name: str):
    return os.environ.get(name)


@dataclass
class Config:
    # --- reference keys (config.go:13-41) ---
    port: int = field(default=8080, metadata={"env": "PORT"})
    log_level: str = field(default="info", metadata={"env": "LOG_LEVEL"})
    max_upload_size: int = field(default=10485760, metadata={"env": "MAX_UPLOAD_SIZE"})
    store_provider: str = field(default="sqlite", metadata={"env": "STORE_PROVIDER"})
    db_host: str = field(default="localhost", metadata={"env": "DB_HOST"})
    db_port: int = field(default=5432, metadata={"env": "DB_PORT"})
    db_user: str = field(default="", metadata={"env": "DB_USER"})
    db_password: str = field(default="", metadata={"env": "DB_PASSWORD"})
    db_name: str = field(default="", metadata={"env": "DB_NAME"})
    queue_provider: str = field(default="broker", metadata={"env": "QUEUE_PROVIDER"})
    queue_url: str = field(default="", metadata={"env": "QUEUE_URL"})
    llm_provider: str = field(default="local", metadata={"env": "LLM_PROVIDER"})
    openai_api_key: str = field(default="", metadata={"env": "OPENAI_API_KEY"})
    llm_model: str = field(default="phi3-mini", metadata={"env": "LLM_MODEL"})
    embedding_model: str = field(default="bge-base", metadata={"env": "EMBEDDING_MODEL"})
    cache_provider: str = field(default="kv", metadata={"env": "CACHE_PROVIDER"})
    redis_addr: str = field(default="localhost:6379", metadata={"env": "REDIS_ADDR"})
    redis_password: str = field(default="", metadata={"env": "REDIS_PASSWORD"})
    cache_ttl: int = field(default=86400, metadata={"env": "CACHE_TTL"})
    # --- new keys: storage / providers ---
    data_dir: str = field(default="./data", metadata={"env": "DATA_DIR"})
    db_path: str = field(default="", metadata={"env": "DB_PATH"})
    embedder_provider: str = field(default="", metadata={"env": "EMBEDDER_PROVIDER"})  # "" -> follow LLM_PROVIDER
    engine_url: str = field(default="", metadata={"env": "ENGINE_URL"})
    query_service_url: str = field(default="http://127.0.0.1:8081/api/query", metadata={"env": "QUERY_SERVICE_URL"})
    # --- new keys: models / numerics ---
    embed_arch: str = field(default="bge-base", metadata={"env": "EMBED_ARCH"})
    llm_arch: str = field(default="phi3-mini", metadata={"env": "LLM_ARCH"})
    embed_dim: int = field(default=0, metadata={"env": "EMBED_DIM"})  # 0 -> encoder hidden size
    dtype: str = field(default="bf16", metadata={"env": "DTYPE"})
    tp_size: int = field(default=1, metadata={"env": "TP_SIZE"})
    index_shards: int = field(default=1, metadata={"env": "INDEX_SHARDS"})
    index_kind: str = field(default="flat", metadata={"env": "INDEX_KIND"})
    ivf_lists: int = field(default=100, metadata={"env": "IVF_LISTS"})
    ivf_probes: int = field(default=1, metadata={"env": "IVF_PROBES"})
    min_similarity: float = field(default=0.7, metadata={"env": "MIN_SIMILARITY"})
    chunk_max_tokens: int = field(default=400, metadata={"env": "CHUNK_MAX_TOKENS"})
    chunk_overlap: int = field(default=80, metadata={"env": "CHUNK_OVERLAP"})
    max_new_tokens: int = field(default=64, metadata={"env": "MAX_NEW_TOKENS"})
    summary_max_new_tokens: int = field(default=128, metadata={"env": "SUMMARY_MAX_NEW_TOKENS"})
    temperature: float = field(default=0.2, metadata={"env": "LLM_TEMPERATURE"})
    weights_path: str = field(default="", metadata={"env": "WEIGHTS_PATH"})
    seed: int = field(default=0, metadata={"env": "SEED"})
    # decode rows of an engine replica; 0 = auto: the largest power of two <= 128 whose KV cache fits
    # KV_CACHE_GB (0: the free HBM after the weights less 48 GB). Deploy stack, 128 in flight:
    # 128 rows 40.6 q/s vs 64 rows 38.3 (profiles/r6/stack)
    max_batch: int = field(default=0, metadata={"env": "ENGINE_MAX_BATCH"})
    kv_cache_gb: float = field(default=0.0, metadata={"env": "KV_CACHE_GB"})  # 0 -> auto
    fault_spec: str = field(default="", metadata={"env": "DA_FAULT"})
    # --- new keys: engine supervision / observability ---
    engine_step_timeout: float = field(default=300.0, metadata={"env": "ENGINE_STEP_TIMEOUT"})
    engine_hard_timeout: float = field(default=0.0, metadata={"env": "ENGINE_HARD_TIMEOUT"})  # 0 -> never exit
    engine_liveness_s: float = field(default=30.0, metadata={"env": "ENGINE_LIVENESS_INTERVAL"})
    engine_metrics_port: int = field(default=0, metadata={"env": "ENGINE_METRICS_PORT"})  # 0 -> off
    worker_concurrency: int = field(default=0, metadata={"env": "WORKER_CONCURRENCY"})  # 0 -> auto
    engine_continuous: bool = field(default=True, metadata={"env": "ENGINE_CONTINUOUS"})
    # decode steps per scheduler tick: 1 lets queued embeds / searches / admissions in between every
    # step (deploy stack, 64 in flight: 35.0 / 34.7 / 33.5 / 32.0 q/s at 1 / 2 / 4 / 8, profiles/r2/stack)
    engine_cb_steps: int = field(default=1, metadata={"env": "ENGINE_CB_STEPS"})
    # decode steps per tick when no request waits for admission (latency of an unloaded request)
    engine_cb_max_steps: int = field(default=16, metadata={"env": "ENGINE_CB_MAX_STEPS"})
    # CUs reserved for the latency lanes (query embeds + search plane); 0 = no partition
    engine_latency_cus: int = field(default=0, metadata={"env": "ENGINE_LATENCY_CUS"})
    # the decode scheduler pauses between steps while question embeds run on the fast lane (their
    # ~100 encoder launches then find free CUs instead of queueing behind decode replays)
    engine_fast_yield: bool = field(default=False, metadata={"env": "ENGINE_FAST_YIELD"})
    # Python GIL switch interval of the engine process (ms; 0 = interpreter default 5 ms). 0.5 ms
    # measured no better for the query path under load (profiles/r3/stack/*switch*)
    engine_switch_interval_ms: float = field(default=0.0, metadata={"env": "ENGINE_SWITCH_INTERVAL_MS"})
    engine_admit_tokens: int = field(default=0, metadata={"env": "ENGINE_ADMIT_TOKENS"})  # 0 -> 4 prefill chunks
    # grouped admission under load (engine/server.py _admit_ready): while >= ENGINE_ADMIT_HOLD_FRAC of
    # the decode rows are busy, arrivals wait until ENGINE_ADMIT_MIN of them (or the free rows) are
    # ready, or the oldest waited ENGINE_ADMIT_WAIT_MS; ENGINE_ADMIT_MIN=1 admits every arrival at once
    engine_admit_min: int = field(default=16, metadata={"env": "ENGINE_ADMIT_MIN"})
    engine_admit_wait_ms: float = field(default=150.0, metadata={"env": "ENGINE_ADMIT_WAIT_MS"})
    engine_admit_hold_frac: float = field(default=0.25, metadata={"env": "ENGINE_ADMIT_HOLD_FRAC"})
    # serving search transport over the sharded index: "plane" (point to point to the owner shards,
    # failures isolated per shard; parallel/search_plane.py) or "rccl" (lock-step rounds of RCCL
    # all-gathers over xGMI; parallel/collective_plane.py; TP_SIZE=1 only)
    search_transport: str = field(default="plane", metadata={"env": "SEARCH_TRANSPORT"})
    search_round_idle_ms: float = field(default=2.0, metadata={"env": "SEARCH_ROUND_IDLE_MS"})
    # an idle collective transport backs off from SEARCH_ROUND_IDLE_MS to this between control
    # gathers (<= 1000 / this gathers per second per rank while nothing is searched)
    search_round_idle_max_ms: float = field(default=50.0, metadata={"env": "SEARCH_ROUND_IDLE_MAX_MS"})
    # --- new keys: durable vector shards (index/wal.py) ---
    index_dir: str = field(default="", metadata={"env": "INDEX_DIR"})  # "" -> DATA_DIR/index; "none" -> off
    index_checkpoint_s: float = field(default=300.0, metadata={"env": "INDEX_CHECKPOINT_S"})
    # startup sweep: a "processing" document younger than this is in flight, not stuck
    sweep_stuck_after_s: float = field(default=600.0, metadata={"env": "SWEEP_STUCK_AFTER_S"})
    index_fsync: bool = field(default=True, metadata={"env": "INDEX_FSYNC"})

    def database_url(self) -> str:
        """config.go:56-64 (kept for parity; the sqlite store uses db_path)."""
        return (f"postgres://{self.db_user}:{self.db_password}@{self.db_host}:{self.db_port}/"
                f"{self.db_name}?sslmode=disable")

    def sqlite_path(self) -> str:
        if self.db_path:
            return self.db_path
        return os.path.join(self.data_dir, "docagents.sqlite3")

    def index_dir_path(self) -> str:
        return self.index_dir or os.path.join(self.data_dir, "index")

    def effective_embedder_provider(self) -> str:
        # reference quirk: embedder chosen by LLM_PROVIDER (internal/app/deps.go:239); an explicit
        # EMBEDDER_PROVIDER overrides it here.
        return self.embedder_provider or self.llm_provider

    def replace(self, **kw) -> "Config":
        return dataclasses.replace(self, **kw)

    # engine compute dtypes (the encoder's; the decoder is bf16): bf16 everywhere; fp16 encoder
    # (f16 MFMA GEMMs + flash, fp16 LayerNorm: BASELINE config 4); fp8 (OCP e4m3) encoder GEMMs.
    # Anything else is refused at startup, never run as something else.
    ENGINE_DTYPES = ("bf16", "fp16", "fp8")

    def validate_engine(self) -> "Config":
        """Startup check of the engine keys whose wrong value would otherwise silently run a
        different configuration (the engine process calls it before touching the GPU)."""
        if self.dtype not in self.ENGINE_DTYPES:
            raise ValueError(f"DTYPE={self.dtype!r} is not supported (choose one of {', '.join(self.ENGINE_DTYPES)})")
        if self.index_kind not in ("flat", "ivfflat"):
            raise ValueError(f"INDEX_KIND={self.index_kind!r} is not supported (flat | ivfflat)")
        if self.tp_size < 1:
            raise ValueError(f"TP_SIZE={self.tp_size} must be >= 1")
        if self.search_transport not in ("plane", "rccl"):
            raise ValueError(f"SEARCH_TRANSPORT={self.search_transport!r} is not supported (plane | rccl)")
        if self.search_transport == "rccl" and self.tp_size > 1:
            # the rounds' RCCL calls run on their own thread; with TP the GPU thread drives the TP
            # communicator at the same time (two communicators from two threads can deadlock)
            raise ValueError("SEARCH_TRANSPORT=rccl needs TP_SIZE=1")
        return self


def load(environ: dict | None = None) -> Config:
    env = os.environ if environ is None else environ
    cfg = Config()
    for f in fields(Config):
        key = f.metadata.get("env")
        if not key or key not in env:
            continue
        raw = env[key]
        try:
            if f.type in ("int", int):
                val = int(raw)
            elif f.type in ("float", float):
                val = float(raw)
            elif f.type in ("bool", bool):  # caarlos0/env uses strconv.ParseBool
                lo = raw.strip().lower()
                if lo not in ("1", "t", "true", "0", "f", "false"):
                    raise ValueError(f"invalid bool {raw!r}")
                val = lo in ("1", "t", "true")
            else:
                val = raw
        except ValueError as e:
            _log.warning("failed to parse env; using defaults where set", extra={"key": key, "err": str(e)})
            continue
        setattr(cfg, f.name, val)
    return cfg
