"""Sliding-window word chunker (internal/chunker/chunker.go:22-57).

Semantics kept bit-exact: tokens are whitespace-delimited words (Go ``strings.Fields``: Unicode
whitespace), MaxTokens <= 0 -> 400, Overlap < 0 -> 0, step = MaxTokens - Overlap (or MaxTokens if
that is <= 0), chunk text = words joined by one space, TokenCount = word count, stop after the
chunk that reaches the last word. A native C++ fast path (``docagents_amd.native``) is used when
built; this module is the reference implementation and the fallback.
"""
from __future__ import annotations

from dataclasses import dataclass

from .preprocess import go_fields


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
    """Go's strings.Fields (unicode.IsSpace; not U+001C..U+001F, which str.split() would cut at)."""
    return go_fields(text)


def chunk_text(text: str, opts: Options | None = None) -> list[Chunk]:
    opts = opts or Options()
    if len(text) > 65536 and text.isascii():
        try:
            return chunk_text_native(text, opts)
        except Exception:  # noqa: BLE001 - native library unavailable: pure-Python path below
            pass
    words = fields(text)
    return [Chunk(index=i, text=" ".join(words[s:e]), token_count=e - s)
            for i, (s, e) in enumerate(chunk_spans(len(words), opts.max_tokens, opts.overlap))]


def chunk_text_native(text: str, opts: Options | None = None) -> list[Chunk]:
    """C++ fast path (docagents_amd/native/textfast.cpp) for ASCII text; identical output."""
    import ctypes

    import numpy as np

    from ..native import textlib
    opts = opts or Options()
    if not text.isascii():
        return chunk_text(text, opts)
    L = textlib()
    b = text.encode("ascii")
    cap = len(b) // 2 + 1
    words = np.empty(2 * cap, dtype=np.int64)
    nw = L.da_word_offsets(b, len(b), words.ctypes.data, cap)
    if nw == 0:
        return []
    mx = opts.max_tokens if opts.max_tokens > 0 else 400
    step = mx - max(0, opts.overlap)
    if step <= 0:
        step = mx
    nchunks = (max(0, nw - mx) + step - 1) // step + 1
    out = ctypes.create_string_buffer(len(b) * (mx // step + 2) + 16)
    meta = np.empty(3 * nchunks + 3, dtype=np.int64)
    nc = L.da_chunk(b, len(b), words.ctypes.data, nw, opts.max_tokens, opts.overlap, out, len(out), meta.ctypes.data,
                    nchunks + 1)
    if nc < 0:
        raise RuntimeError("native chunker buffer too small")
    raw = out.raw
    return [Chunk(index=i, text=raw[meta[3 * i]:meta[3 * i] + meta[3 * i + 1]].decode("ascii"),
                  token_count=int(meta[3 * i + 2])) for i in range(nc)]
