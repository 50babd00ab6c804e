"""Deterministic cache keys, bit-exact with internal/cache/cache.go:51-74.

``generate_cache_key``: doc ids sorted as byte strings (Go string ``>``), ``sha256("q:%s|docs:%s|k:%d")``
hex. ``generate_embedding_key``: ``sha256(text)`` hex. Redis-style prefixes ``query:`` / ``embed:``
(internal/cache/redis.go:12-18).
"""
from __future__ import annotations

import hashlib

QUERY_PREFIX = "query:"
EMBED_PREFIX = "embed:"


def generate_cache_key(question: str, doc_ids: list[str], top_k: int) -> str:
    ids = sorted(doc_ids, key=lambda s: s.encode("utf-8"))
    data = f"q:{question}|docs:{','.join(ids)}|k:{top_k}"
    return hashlib.sha256(data.encode("utf-8")).hexdigest()


def generate_embedding_key(text: str) -> str:
    return hashlib.sha256(text.encode("utf-8")).hexdigest()
