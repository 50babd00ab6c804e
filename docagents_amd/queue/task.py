"""Task envelope and queue contract (internal/queue/queue.go:13-56).

Wire format is the reference's Go JSON of ``queue.Task`` (no json tags): ``{"ID": uuid,
"Type": "parse"|"analyze", "Payload": base64(payload JSON), "Attempts": n, "MaxAttempts": n,
"NotBefore": RFC3339Nano}`` — so a Go worker and a Python worker can share one broker.
Subjects ``tasks.<type>``, queue groups ``workers-<type>`` (internal/queue/nats.go:37-43).
"""
from __future__ import annotations

import asyncio
import base64
import datetime as dt
import json
import re
import uuid
from dataclasses import dataclass, field
from typing import Awaitable, Callable, Protocol

from ..utils.retry import exponential_backoff

_TIME_RE = re.compile(r"^(\d{4}-\d\d-\d\dT\d\d:\d\d:\d\d)(\.\d+)?(Z|[+-]\d\d:\d\d)$")
TASK_PARSE = "parse"
TASK_ANALYZE = "analyze"
ZERO_TIME = "0001-01-01T00:00:00Z"


def subject_for(task_type: str) -> str:
    return "tasks." + task_type


def group_for(task_type: str) -> str:
    return "workers-" + task_type


def _fmt_time(t: dt.datetime | None) -> str:
    if t is None:
        return ZERO_TIME
    t = t.astimezone(dt.timezone.utc)
    s = t.strftime("%Y-%m-%dT%H:%M:%S")
    if t.microsecond:
        s += ("." + f"{t.microsecond:06d}").rstrip("0")
    return s + "Z"


def _parse_time(s: str | None) -> dt.datetime | None:
    if not s or s.startswith("0001-01-01"):
        return None
    m = _TIME_RE.match(s)
    if not m:
        raise ValueError(f"bad time {s!r}")
    base, frac, tz = m.groups()
    frac = ((frac or ".")[1:] + "000000")[:6]  # Go may emit nanoseconds; keep microseconds
    tz = "+00:00" if tz == "Z" else tz
    return dt.datetime.fromisoformat(f"{base}.{frac}{tz}")


@dataclass
class Task:
    type: str
    payload: bytes = b""
    id: str = ""
    attempts: int = 0
    max_attempts: int = 0
    not_before: dt.datetime | None = None
    trace_id: str = ""          # extension: propagated request id
    extra: dict = field(default_factory=dict)

    def encode(self) -> bytes:
        d = {"ID": self.id or str(uuid.UUID(int=0)), "Type": self.type,
             "Payload": base64.b64encode(self.payload).decode() if self.payload else None,
             "Attempts": self.attempts, "MaxAttempts": self.max_attempts, "NotBefore": _fmt_time(self.not_before)}
        if self.trace_id:
            d["TraceID"] = self.trace_id
        return json.dumps(d, separators=(",", ":")).encode()

    @classmethod
    def decode(cls, data: bytes) -> "Task":
        d = json.loads(data)
        p = d.get("Payload")
        return cls(type=d.get("Type", ""), payload=base64.b64decode(p) if p else b"", id=d.get("ID", ""),
                   attempts=int(d.get("Attempts", 0)), max_attempts=int(d.get("MaxAttempts", 0)),
                   not_before=_parse_time(d.get("NotBefore")), trace_id=d.get("TraceID", ""))

    def payload_json(self):
        return json.loads(self.payload or b"null")


Handler = Callable[[Task], Awaitable[None]]


class Queue(Protocol):
    async def enqueue(self, task: Task) -> None: ...

    async def worker(self, task_type: str, handler: Handler, stop: asyncio.Event | None = None) -> None: ...


class QueueError(RuntimeError):
    pass


async def enqueue_with_retry(q: Queue, task: Task, attempts: int, base: float) -> None:
    """internal/queue/queue.go:39-56: try ``attempts`` times, sleeping base*2^attempt between tries."""
    if attempts <= 0:
        attempts = 1
    for attempt in range(attempts):
        try:
            await q.enqueue(task)
            return
        except Exception:
            if attempt == attempts - 1:
                raise
        await asyncio.sleep(exponential_backoff(attempt, base))


def prepare_for_publish(task: Task) -> Task:
    """nats.go:26-33: assign an ID, require a Type."""
    if not task.type:
        raise QueueError("task type required")
    if not task.id or task.id == str(uuid.UUID(int=0)):
        task.id = str(uuid.uuid4())
    return task


def next_retry(task: Task, now: dt.datetime | None = None) -> Task | None:
    """nats.go:69-83: Attempts++, MaxAttempts defaults to 5, NotBefore = now + 1s*2^Attempts;
    None when the task is permanently failed."""
    task.attempts += 1
    if task.max_attempts == 0:
        task.max_attempts = 5
    if task.attempts < task.max_attempts:
        now = now or dt.datetime.now(dt.timezone.utc)
        task.not_before = now + dt.timedelta(seconds=exponential_backoff(task.attempts, 1.0))
        return task
    return None
