"""Text helpers with reference-exact semantics.

* ``preprocess_text`` — internal/embeddings/openai.go:131-142: strip ``[\\x00-\\x08\\x0B-\\x0C\\x0E-\\x1F\\x7F]``,
  TrimSpace (Unicode), then collapse RE2 ``\\s+`` (ASCII ``[\\t\\n\\f\\r ]`` only — RE2's \\s is ASCII and
  excludes \\v) to one space.
* ``truncate_preview`` — cmd/query/main.go:186-195: byte-length cut at 150 with a word-boundary
  backoff; operates on UTF-8 BYTES like Go slicing (may split a rune). The bytes of a split rune
  come back as lone surrogates, one per byte (``surrogateescape``), so the Go JSON writer
  (api/gojson.py) emits one ``\\ufffd`` escape per invalid byte, as Go's ``encoding/json`` does.
* ``extract_summary`` — internal/llm/openai.go:127-144 (``strings.TrimSpace``: Go's whitespace).
* ``go_fields`` / ``go_trim_space`` — Go's ``strings.Fields`` / ``strings.TrimSpace``: whitespace is
  ``unicode.IsSpace``, which unlike Python's ``str.isspace`` excludes U+001C..U+001F.
"""
from __future__ import annotations

import re

_CTRL = re.compile(r"[\x00-\x08\x0B-\x0C\x0E-\x1F\x7F]")
# unicode.IsSpace: '\t', '\n', '\v', '\f', '\r', ' ', U+0085, U+00A0 and the White_Space property
GO_SPACE = "\t\n\v\f\r \x85\xa0\u1680\u2000\u2001\u2002\u2003\u2004\u2005\u2006\u2007\u2008\u2009\u200a" \
           "\u2028\u2029\u202f\u205f\u3000"
_GO_SPACE_RUN = re.compile(f"[{GO_SPACE}]+")
_PY_ONLY_SPACE = ("\x1c", "\x1d", "\x1e", "\x1f")  # str.isspace() but not unicode.IsSpace


def go_fields(text: str) -> list[str]:
    """strings.Fields: maximal runs of non-whitespace (unicode.IsSpace). ``str.split()`` is the
    same split except for U+001C..U+001F, which only Python counts as whitespace."""
    if not any(c in text for c in _PY_ONLY_SPACE):
        return text.split()
    return [w for w in _GO_SPACE_RUN.split(text) if w]


def go_trim_space(text: str) -> str:
    """strings.TrimSpace (unicode.IsSpace at both ends)."""
    return text.strip(GO_SPACE)


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
        return b[:idx].decode("utf-8", errors="surrogateescape") + "..."
    return head.decode("utf-8", errors="surrogateescape") + "..."


def extract_summary(content: str) -> tuple[str, list[str]]:
    points: list[str] = []
    summary_lines: list[str] = []
    for line in content.split("\n"):
        trimmed = go_trim_space(line)
        if not trimmed:
            continue
        if trimmed.startswith("-") or trimmed.startswith("*"):
            points.append(trimmed.lstrip("-* "))
        else:
            summary_lines.append(trimmed)
    return " ".join(summary_lines), points
