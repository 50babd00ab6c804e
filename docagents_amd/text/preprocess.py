"""Text helpers with reference-exact semantics.

* ``preprocess_text`` — internal/embeddings/openai.go:131-142: strip ``[\\x00-\\x08\\x0B-\\x0C\\x0E-\\x1F\\x7F]``,
  TrimSpace (Unicode), then collapse RE2 ``\\s+`` (ASCII ``[\\t\\n\\f\\r ]`` only — RE2's \\s is ASCII and
  excludes \\v) to one space.
* ``truncate_preview`` — cmd/query/main.go:186-195: byte-length cut at 150 with a word-boundary
  backoff; operates on UTF-8 BYTES like Go slicing (may split a rune; decoded with replacement).
* ``extract_summary`` — internal/llm/openai.go:127-144.
"""
from __future__ import annotations

import re

_CTRL = re.compile(r"[\x00-\x08\x0B-\x0C\x0E-\x1F\x7F]")
_WS = re.compile(r"[\t\n\f\r ]+")


def preprocess_text(text: str) -> str:
    text = _CTRL.sub("", text)
    text = text.strip()
    return _WS.sub(" ", text)


def truncate_preview(s: str, max_len: int = 150) -> str:
    b = s.encode("utf-8")
    if len(b) <= max_len:
        return s
    head = b[:max_len]
    idx = head.rfind(b" ")
    if idx > 0:
        return b[:idx].decode("utf-8", errors="replace") + "..."
    return head.decode("utf-8", errors="replace") + "..."


def extract_summary(content: str) -> tuple[str, list[str]]:
    points: list[str] = []
    summary_lines: list[str] = []
    for line in content.split("\n"):
        trimmed = line.strip()
        if not trimmed:
            continue
        if trimmed.startswith("-") or trimmed.startswith("*"):
            points.append(trimmed.lstrip("-* "))
        else:
            summary_lines.append(trimmed)
    return " ".join(summary_lines), points
