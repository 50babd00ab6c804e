"""Structured JSON logging with the reference's schema and level parsing.

Reference: internal/logger/logger.go:9-26 (slog JSON handler to stdout; "debug"/"warn"/"error",
anything else -> info). Records are one JSON object per line: ``time``, ``level``, ``msg`` and the
key/value attributes, as slog's JSONHandler writes them.
"""
from __future__ import annotations

import datetime as _dt
import json
import logging
import sys
import threading

_LEVELS = {"debug": logging.DEBUG, "warn": logging.WARNING, "error": logging.ERROR}
_SLOG_NAMES = {logging.DEBUG: "DEBUG", logging.INFO: "INFO", logging.WARNING: "WARN", logging.ERROR: "ERROR",
               logging.CRITICAL: "ERROR"}


def parse_level(level: str) -> int:
    return _LEVELS.get(level, logging.INFO)


class Logger:
    """A tiny slog-like logger: ``log.info("msg", "k1", v1, "k2", v2)`` or ``log.info("msg", k=v)``."""

    def __init__(self, level: int = logging.INFO, stream=None, attrs: dict | None = None):
        self.level = level
        self.stream = stream if stream is not None else sys.stdout
        self.attrs = dict(attrs or {})
        self._lock = threading.Lock()

    def with_(self, *kv, **kw) -> "Logger":
        a = dict(self.attrs)
        a.update(_kv(kv, kw))
        lg = Logger(self.level, self.stream, a)
        lg._lock = self._lock
        return lg

    def enabled(self, lvl: int) -> bool:
        return lvl >= self.level

    def _emit(self, lvl: int, msg: str, kv, kw):
        if lvl < self.level:
            return
        rec = {"time": _dt.datetime.now(_dt.timezone.utc).astimezone().isoformat(timespec="microseconds"),
               "level": _SLOG_NAMES.get(lvl, "INFO"), "msg": msg}
        rec.update(self.attrs)
        rec.update(_kv(kv, kw))
        line = json.dumps(rec, default=str, ensure_ascii=False)
        with self._lock:
            try:
                self.stream.write(line + "\n")
                self.stream.flush()
            except ValueError:  # closed stream during interpreter shutdown
                pass

    def debug(self, msg, *kv, **kw):
        self._emit(logging.DEBUG, msg, kv, kw)

    def info(self, msg, *kv, **kw):
        self._emit(logging.INFO, msg, kv, kw)

    def warn(self, msg, *kv, **kw):
        self._emit(logging.WARNING, msg, kv, kw)

    warning = warn

    def error(self, msg, *kv, **kw):
        self._emit(logging.ERROR, msg, kv, kw)


def _kv(kv, kw) -> dict:
    out = {}
    it = list(kv)
    for i in range(0, len(it) - 1, 2):
        out[str(it[i])] = _val(it[i + 1])
    if len(it) % 2:
        out["!BADKEY"] = _val(it[-1])
    for k, v in kw.items():
        out[k] = _val(v)
    return out


def _val(v):
    if isinstance(v, BaseException):
        return str(v)
    return v


def new(level: str = "info", stream=None) -> Logger:
    return Logger(parse_level(level), stream)


def discard() -> Logger:
    import io
    return Logger(logging.CRITICAL + 10, io.StringIO())
