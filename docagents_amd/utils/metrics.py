"""Prometheus metrics shared by the agents, queue workers and the engine.

The reference exports no metrics at all (README.md:706-710); everything here is new. Metrics are
created once per process; when ``prometheus_client`` is missing every metric is a no-op object so
callers never branch.
"""
from __future__ import annotations

import time


class _Noop:
    def labels(self, *a, **k):
        return self

    def inc(self, *a, **k):
        pass

    def observe(self, *a, **k):
        pass

    def set(self, *a, **k):
        pass


_made: dict[str, object] = {}


def _metric(kind: str, name: str, doc: str, labels=(), **kw):
    if name in _made:
        return _made[name]
    try:
        import prometheus_client as pc
        m = getattr(pc, kind)(name, doc, list(labels), **kw)
    except ValueError:  # already registered (module reloaded in tests)
        import prometheus_client as pc
        m = pc.REGISTRY._names_to_collectors.get(name) or _Noop()  # noqa: SLF001
    except Exception:  # noqa: BLE001 - prometheus_client absent
        m = _Noop()
    _made[name] = m
    return m


_LAT = (0.0005, 0.001, 0.005, 0.01, 0.025, 0.05, 0.1, 0.25, 0.5, 1, 2.5, 5, 10, 30, 60, 120)

# queue workers (internal/queue/nats.go:53-83 semantics)
TASKS = _metric("Counter", "da_tasks_total", "queue tasks by outcome", ["type", "outcome"])
TASK_SECONDS = _metric("Histogram", "da_task_seconds", "handler latency per task attempt", ["type"], buckets=_LAT)
TASK_ATTEMPTS = _metric("Histogram", "da_task_attempts", "attempt number at which a task finished", ["type"],
                        buckets=(1, 2, 3, 4, 5, 6, 8, 10))

# engine (one series set per engine process / rank 0)
ENGINE_BATCHES = _metric("Counter", "da_engine_batches_total", "engine micro-batches executed", ["method"])
ENGINE_ITEMS = _metric("Counter", "da_engine_items_total", "items processed by the engine", ["method"])
ENGINE_BATCH_SIZE = _metric("Histogram", "da_engine_batch_items", "items per engine micro-batch", ["method"],
                            buckets=(1, 2, 4, 8, 16, 32, 64, 128, 256, 512, 1024))
ENGINE_STEP = _metric("Histogram", "da_engine_step_seconds", "engine command wall time", ["cmd"], buckets=_LAT)
ENGINE_TOKENS = _metric("Counter", "da_engine_tokens_total", "tokens processed by the decoder", ["phase"])
ENGINE_COLLECTIVE = _metric("Counter", "da_engine_collective_seconds_total", "time inside collectives", ["op"])
ENGINE_INDEX_ROWS = _metric("Gauge", "da_engine_index_rows", "vector index rows per shard", ["rank"])
ENGINE_HBM = _metric("Gauge", "da_engine_hbm_bytes", "device memory in use", ["rank", "kind"])
ENGINE_HEALTHY = _metric("Gauge", "da_engine_healthy", "1 when the watchdog sees no stuck step", [])
ENGINE_EMBED_TRUNCATED = _metric("Counter", "da_engine_embed_truncated_total",
                                 "encoder inputs cut at the max position (512): texts and tokens dropped", ["what"])
ENGINE_LIVE_RANKS = _metric("Gauge", "da_engine_live_ranks", "ranks answering the last liveness all-reduce", [])


class timer:
    """``with timer(hist.labels(x)):`` observes elapsed seconds."""

    def __init__(self, h):
        self.h = h

    def __enter__(self):
        self.t0 = time.perf_counter()
        return self

    def __exit__(self, *exc):
        self.elapsed = time.perf_counter() - self.t0
        self.h.observe(self.elapsed)
        return False
