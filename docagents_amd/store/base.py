"""Domain types and the persistence contract (internal/store/store.go:13-67)."""
from __future__ import annotations

import datetime as dt
from dataclasses import dataclass, field
from typing import Protocol

STATUS_PROCESSING = "processing"
STATUS_READY = "ready"
STATUS_FAILED = "failed"


class SummaryNotFound(LookupError):
    """ErrSummaryNotFound (store.go:21)."""

    def __str__(self):
        return "summary not found"


class DocumentNotFound(LookupError):
    def __str__(self):
        return "document not found"


@dataclass
class Document:
    id: str
    filename: str
    status: str = STATUS_PROCESSING
    created_at: dt.datetime | None = None
    seq: int = 0  # dense integer id (doc slot)


@dataclass
class Chunk:
    id: str = ""
    document_id: str = ""
    index: int = 0
    text: str = ""
    token_count: int = 0
    key: int = 0  # integer vector id in the HBM index


@dataclass
class Summary:
    document_id: str = ""
    summary: str = ""
    key_points: list[str] = field(default_factory=list)


@dataclass
class Embedding:
    chunk_id: str
    vector: object  # np.ndarray / list[float] / torch.Tensor
    model: str = ""


@dataclass
class SearchResult:
    chunk: Chunk
    score: float
    summary: Summary
    # the chunk's decoder token ids (int32 bytes, None: never tokenized) when the store read them
    # with the hit (tokens_loaded), so the Answer prompt needs no second lookup
    tokens: bytes | None = None
    tokens_loaded: bool = False


class Store(Protocol):
    async def create_document(self, filename: str) -> Document: ...
    async def get_document(self, doc_id: str) -> Document: ...
    async def update_document_status(self, doc_id: str, status: str) -> None: ...
    async def save_chunks(self, doc_id: str, chunks: list[Chunk]) -> list[Chunk]: ...
    async def list_chunks(self, doc_id: str) -> list[Chunk]: ...
    async def save_summary(self, doc_id: str, summary: Summary) -> None: ...
    async def save_embeddings(self, embs: list[Embedding]) -> None: ...
    async def get_summary(self, doc_id: str) -> Summary: ...
    async def top_k(self, doc_ids: list[str], vector, k: int) -> list[SearchResult]: ...
