"""In-HBM vector indexes (flat brute force, IVFFlat) — the pgvector replacement."""
from __future__ import annotations


def make_index(kind: str, dim: int, device, lists: int = 100, probes: int = 1, capacity: int = 1024):
    if kind == "flat":
        from .flat import FlatIndex
        return FlatIndex(dim, device, capacity=capacity)
    if kind == "ivfflat":
        from .ivf import IVFFlatIndex
        return IVFFlatIndex(dim, device, lists=lists, probes=probes, capacity=capacity)
    raise ValueError(f"unknown INDEX_KIND {kind!r} (flat | ivfflat)")
