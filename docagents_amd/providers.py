"""Embedder and LLM providers (the ports of internal/embeddings/embeddings.go:7-10 and
internal/llm/llm.go:6-9).

* ``stub``   — deterministic, CPU-only: hash-seeded unit vectors / canned text. Makes the
               reference's ``LLM_PROVIDER=stub`` actually buildable (Appendix B #12).
* ``local``  — the MI355X engine in this process (``docagents_amd.engine.engine.Engine``).
* ``engine`` — the engine server over RPC (``docagents_amd.engine.rpc``); concurrent requests
               from all agents are micro-batched there into one encoder / decoder launch.
"""
from __future__ import annotations

import os

import asyncio
import hashlib

import numpy as np

from .text.preprocess import extract_summary, preprocess_text


class EmbedError(RuntimeError):
    pass


# ------------------------------------------------------------------------------ embedders
class StubEmbedder:
    """Hash-seeded random unit vectors of ``dim`` (same text -> same vector)."""

    def __init__(self, dim: int = 768):
        self.dim = dim

    def _vec(self, text: str) -> np.ndarray:
        seed = int.from_bytes(hashlib.sha256(text.encode()).digest()[:8], "little")
        v = np.random.default_rng(seed).standard_normal(self.dim).astype(np.float32)
        return v / np.linalg.norm(v)

    async def embed(self, text: str) -> np.ndarray:
        t = preprocess_text(text)
        if not t:
            raise EmbedError("text is empty after preprocessing")
        return self._vec(t)

    async def embed_batch(self, texts: list[str]) -> list[np.ndarray]:
        # 1:1 with the input (the reference drops empty texts and then mis-indexes)
        return [self._vec(preprocess_text(t)) for t in texts]


class LocalEmbedder:
    def __init__(self, engine):
        self.engine = engine

    async def embed(self, text: str) -> np.ndarray:
        t = preprocess_text(text)
        if not t:
            raise EmbedError("text is empty after preprocessing")
        v = await asyncio.to_thread(self.engine.embed, [t], False)
        return v[0].float().cpu().numpy()

    async def embed_batch(self, texts: list[str]) -> list[np.ndarray]:
        if not texts:
            return []
        v = await asyncio.to_thread(self.engine.embed, texts)
        return list(v.float().cpu().numpy())


class RemoteEmbedder:
    def __init__(self, client):
        self.client = client

    async def embed(self, text: str) -> np.ndarray:
        t = preprocess_text(text)
        if not t:
            raise EmbedError("text is empty after preprocessing")
        r = await self.client.call("embed", texts=[t], preprocess=False)
        return r["vecs"][0]

    async def embed_batch(self, texts: list[str]) -> list[np.ndarray]:
        if not texts:
            return []
        r = await self.client.call("embed", texts=list(texts), preprocess=True)
        return list(r["vecs"])


# ------------------------------------------------------------------------------ LLM clients
class StubLLM:
    """Deterministic text; confidence = context quality x 0.9 (a fixed 'mean token probability')."""

    async def summarize(self, text: str):
        words = text.split()
        head = " ".join(words[:30])
        content = f"Summary of {len(words)} words: {head}\n- first point: {' '.join(words[:5])}\n" \
                  f"- second point: {' '.join(words[5:10])}"
        return extract_summary(content)

    async def answer(self, question: str, context: str, quality: float):
        delay = float(os.environ.get("DA_STUB_ANSWER_S", "0") or 0)  # load tests: a model-like answer time
        if delay > 0:
            await asyncio.sleep(delay)
        if not context.strip():
            return "I don't have enough information to answer this question", float(quality) * 0.9
        first = context.strip().split("\n")[0][:200]
        return f"According to the documentation, {first}", float(quality) * 0.9

    async def answer_chunks(self, question: str, chunks, quality: float):
        return await self.answer(question, "".join(t + "\n" for t, _ in chunks), quality)


class LocalLLM:
    supports_chunks = True  # Answer from chunk token ids cached at ingest

    def __init__(self, engine):
        self.engine = engine

    async def summarize(self, text: str):
        return (await asyncio.to_thread(self.engine.summarize_many, [text]))[0]

    async def answer(self, question: str, context: str, quality: float):
        return await asyncio.to_thread(self.engine.answer_text, question, context, quality)

    async def answer_chunks(self, question: str, chunks, quality: float):
        ids = [(tok.tolist() if isinstance(tok, np.ndarray) else tok) if tok is not None else self.engine._ids(txt)
               for txt, tok in chunks]
        return (await asyncio.to_thread(self.engine.answer_many, [(question, ids, quality)]))[0]


class RemoteLLM:
    supports_chunks = True

    def __init__(self, client):
        self.client = client

    async def summarize(self, text: str):
        r = await self.client.call("summarize", texts=[text])
        s, kp = r["results"][0]
        return s, list(kp)

    async def answer(self, question: str, context: str, quality: float):
        r = await self.client.call("answer", items=[{"question": question, "context": context, "quality": quality}])
        a, c = r["results"][0]
        return a, float(c)

    async def answer_chunks(self, question: str, chunks, quality: float):
        item = {"question": question, "quality": quality,
                "chunks": [{"text": t, "tokens": (np.asarray(tok, dtype=np.int32) if tok is not None else None)}
                           for t, tok in chunks]}
        r = await self.client.call("answer", items=[item])
        a, c = r["results"][0]
        return a, float(c)
