"""Vector backends for ``CompositeStore``.

* ``LocalVectors``  — an in-process HBM index (flat or IVFFlat; CPU tensors in tests).
* ``EngineVectors`` — the index lives in the engine server process that owns the GPU(s); vectors
                      travel over the engine RPC (``docagents_amd.engine.rpc``).
Both return ``[(chunk_key, score)]`` sorted by score desc with the similarity floor and the doc
filter applied before top-k (postgres.go:225-243 semantics, exact).
"""
from __future__ import annotations

import asyncio

import numpy as np
import torch


class LocalVectors:
    def __init__(self, index):
        self.index = index
        self.lock = asyncio.Lock()

    async def add(self, doc_id: str, keys: np.ndarray, vecs: np.ndarray):
        t = torch.from_numpy(np.ascontiguousarray(vecs, dtype=np.float32))
        async with self.lock:
            await asyncio.to_thread(self.index.add, doc_id, keys, t)

    async def search(self, vector: np.ndarray, doc_ids: list[str], k: int, min_sim: float):
        q = torch.from_numpy(np.ascontiguousarray(vector, dtype=np.float32)).view(1, -1)

        def f():
            s, rows = self.index.search(q, k, min_sim, [doc_ids])
            s = s[0].float().cpu().numpy()
            keys = self.index.row_ids(rows[0].cpu().numpy().astype(np.int64))
            return [(int(kk), float(sc)) for kk, sc in zip(keys, s) if kk >= 0 and np.isfinite(sc)]
        async with self.lock:
            return await asyncio.to_thread(f)

    async def remove_doc(self, doc_id: str):
        async with self.lock:
            return self.index.remove_doc(doc_id)


class EngineVectors:
    def __init__(self, client):
        self.client = client

    async def add(self, doc_id: str, keys: np.ndarray, vecs: np.ndarray):
        await self.client.call("index_add", doc_id=doc_id, keys=np.asarray(keys, dtype=np.int64),
                               vecs=np.asarray(vecs, dtype=np.float32))

    async def search(self, vector: np.ndarray, doc_ids: list[str], k: int, min_sim: float):
        r = await self.client.call("search", vecs=np.asarray(vector, dtype=np.float32).reshape(1, -1),
                                   filters=[list(doc_ids)], k=int(k), min_sim=float(min_sim))
        keys, scores = r["keys"][0], r["scores"][0]
        return [(int(kk), float(sc)) for kk, sc in zip(keys, scores) if kk >= 0]

    async def embed_search(self, text: str, doc_ids: list[str], k: int, min_sim: float):
        """(question vector, [(chunk_key, score)]) from ONE engine RPC: the engine embeds the text on
        its fast lane and searches every shard through the search plane."""
        r = await self.client.call("embed_search", texts=[text], filters=[list(doc_ids)], k=int(k),
                                   min_sim=float(min_sim), preprocess=False)
        keys, scores = r["keys"][0], r["scores"][0]
        return r["vecs"][0], [(int(kk), float(sc)) for kk, sc in zip(keys, scores) if kk >= 0]

    async def remove_doc(self, doc_id: str):
        return await self.client.call("index_remove", doc_id=doc_id)

    async def embed_index(self, doc_id: str, keys: np.ndarray, texts: list[str]) -> tuple[int, int]:
        """Embed ``texts`` on the engine and write the rows straight into the owner shard (no vector
        bytes leave the GPU). Returns (rows written, dim)."""
        r = await self.client.call("embed_index", doc_id=doc_id, keys=np.asarray(keys, dtype=np.int64),
                                   texts=list(texts))
        return int(r["rows"]), int(r["dim"])

    async def doc_rows(self) -> dict[str, int]:
        """{document id: indexed rows} over every shard (startup sweep)."""
        return dict(await self.client.call("index_docs"))
