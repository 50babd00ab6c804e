"""Fault injection hooks: ``DA_FAULT="site:prob,site2:prob"``.

Sites used by the framework: ``queue.enqueue``, ``handler.parse``, ``handler.analyze``,
``store.save_chunks``, ``engine.embed``, ``engine.generate``, ``cache.get``, ``cache.set``.
``prob`` is 0..1; ``site:n`` with n >= 1 fails the first n calls. Deterministic per process.
"""
from __future__ import annotations

import os
import random
import threading

_lock = threading.Lock()
_spec: dict[str, float] | None = None
_counts: dict[str, int] = {}
_rng = random.Random(int(os.environ.get("DA_FAULT_SEED", "0")))


class InjectedFault(RuntimeError):
    pass


def _load() -> dict[str, float]:
    global _spec
    if _spec is None:
        spec = {}
        for part in filter(None, os.environ.get("DA_FAULT", "").split(",")):
            site, _, p = part.partition(":")
            try:
                spec[site.strip()] = float(p)
            except ValueError:
                pass
        _spec = spec
    return _spec


def configure(spec: str | dict | None):
    global _spec
    with _lock:
        if spec is None:
            _spec = {}
        elif isinstance(spec, dict):
            _spec = dict(spec)
        else:
            os.environ["DA_FAULT"] = spec
            _spec = None
            _load()
        _counts.clear()


_delays: dict[str, float] = {}


def configure_delay(spec: dict | None):
    """Test hook: ``maybe_delay(site)`` sleeps ``spec[site]`` seconds (a slow replica / GPU thread)."""
    with _lock:
        _delays.clear()
        _delays.update(spec or {})


def maybe_delay(site: str):
    d = _delays.get(site)
    if d:
        import time
        time.sleep(d)


def maybe_fail(site: str):
    spec = _load()
    if not spec:
        return
    p = spec.get(site)
    if p is None:
        return
    with _lock:
        n = _counts.get(site, 0)
        _counts[site] = n + 1
        fail = (n < p) if p >= 1 else (_rng.random() < p)
    if fail:
        raise InjectedFault(f"injected fault at {site}")
