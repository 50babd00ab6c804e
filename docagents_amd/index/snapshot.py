"""Index shard snapshot / restore: safetensors with the live rows (removed
documents compacted away), their external ids and doc slots, plus a JSON doc table in the metadata
header. IVF shards also store centroids; lists are rebuilt on load."""
from __future__ import annotations

import json
import os

import numpy as np
import torch
from safetensors.torch import load_file, save_file


def save_index(index, path: str, extra_meta: dict | None = None, durable: bool = True) -> str:
    """Write the snapshot to ``path`` atomically (tmp file + rename); ``durable``: fsync the file
    before the rename and the directory after it, so the snapshot survives a power loss once this
    returns (the vector log deletes the generations it covers right after)."""
    with index.reading():
        sel, docs = index.live_rows_by_doc()
        docs = [[d, n] for d, n in docs]
        selt = torch.from_numpy(sel.astype(np.int64)).to(index.device)
        tensors = {"X": index.X.index_select(0, selt).cpu().contiguous(),
                   "ids": torch.from_numpy(index.ids[sel].copy())}
        if getattr(index, "centroids", None) is not None:
            tensors["centroids"] = index.centroids.cpu().contiguous()
        meta = {"dim": str(index.dim), "kind": index.kind, "docs": json.dumps(docs)}
        meta.update({k: str(v) for k, v in (extra_meta or {}).items()})
    tmp = path + ".tmp"
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    save_file(tensors, tmp, metadata=meta)
    if durable:
        fd = os.open(tmp, os.O_RDONLY)
        try:
            os.fsync(fd)
        finally:
            os.close(fd)
    os.replace(tmp, path)
    if durable:
        dfd = os.open(os.path.dirname(os.path.abspath(path)), os.O_RDONLY)
        try:
            os.fsync(dfd)
        finally:
            os.close(dfd)
    return path


def snapshot_meta(path: str) -> dict:
    from safetensors import safe_open
    with safe_open(path, framework="pt") as f:
        return dict(f.metadata() or {})


def load_index(index, path: str) -> int:
    from safetensors import safe_open
    with safe_open(path, framework="pt") as f:
        meta = f.metadata()
    t = load_file(path)
    if int(meta["dim"]) != index.dim:
        raise ValueError(f"snapshot dim {meta['dim']} != index dim {index.dim}")
    docs = json.loads(meta["docs"])
    X, ids = t["X"], t["ids"].numpy()
    with index.writing():
        index.add_bulk([d for d, _ in docs], [n for _, n in docs], ids, X)
        if "centroids" in t and hasattr(index, "_build_lists"):
            index.centroids = t["centroids"].to(index.device)
            index._build_lists()
    return len(index)
