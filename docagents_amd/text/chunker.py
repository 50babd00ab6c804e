"""Sliding-window word chunker (internal/chunker/chunker.go:22-57).

Semantics kept bit-exact: tokens are whitespace-delimited words (Go ``strings.Fields``: Unicode
whitespace), MaxTokens <= 0 -> 400, Overlap < 0 -> 0, step = MaxTokens - Overlap (or MaxTokens if
that is <= 0), chunk text = words joined by one space, TokenCount = word count, stop after the
chunk that reaches the last word. A native C++ fast path (``docagents_amd.native``) is used when
built; this module is the reference implementation and the fallback.
"""
from __future__ import annotations

from dataclasses import dataclass


@dataclass
class Options:
    max_tokens: int = 400
    overlap: int = 0


@dataclass
class Chunk:
    index: int
    text: str
    token_count: int


def chunk_spans(n_words: int, max_tokens: int, overlap: int) -> list[tuple[int, int]]:
    """[start, end) word ranges produced by ChunkText for a text of ``n_words`` words."""
    if max_tokens <= 0:
        max_tokens = 400
    if overlap < 0:
        overlap = 0
    if n_words == 0:
        return []
    step = max_tokens - overlap
    if step <= 0:
        step = max_tokens
    spans = []
    start = 0
    while start < n_words:
        end = min(start + max_tokens, n_words)
        spans.append((start, end))
        if end == n_words:
            break
        start += step
    return spans


def fields(text: str) -> list[str]:
    # Python's str.split() with no argument splits on Unicode whitespace runs and drops empties,
    # matching Go's strings.Fields (unicode.IsSpace) for all practical inputs.
    return text.split()


def chunk_text(text: str, opts: Options | None = None) -> list[Chunk]:
    opts = opts or Options()
    words = fields(text)
    return [Chunk(index=i, text=" ".join(words[s:e]), token_count=e - s)
            for i, (s, e) in enumerate(chunk_spans(len(words), opts.max_tokens, opts.overlap))]
