"""Per-request event timeline across the stack's processes (load diagnosis; off unless asked).

``DA_REQ_TIMELINE=<dir>``: every process appends JSON lines ``{"e": event, "t": wall time, "pid",
...}`` to ``<dir>/<pid>.jsonl`` — the query service per request (handler start, question embedded,
answer sent / received, reply), the engine per answer / embed_search RPC (receipt, admission
hand-off to the scheduler, reply) and ``bench/loadgen.py`` per request (send, receive).
``bench/timeline_report.py`` joins them by question text (unique per request in a load run) into
where each request spent its time. Wall clock (``time.time()``): every process runs on one box.
"""
from __future__ import annotations

import json
import os
import threading
import time

_DIR = os.environ.get("DA_REQ_TIMELINE", "")
_lock = threading.Lock()
_f = None


def enabled() -> bool:
    return bool(_DIR)


def mark(event: str, **kw) -> None:
    global _f
    if not _DIR:
        return
    rec = {"e": event, "t": time.time(), **kw}
    line = json.dumps(rec, default=str) + "\n"
    with _lock:
        if _f is None:
            os.makedirs(_DIR, exist_ok=True)
            _f = open(os.path.join(_DIR, f"{os.getpid()}.jsonl"), "a", buffering=1)
        _f.write(line)
