"""In-process message bus with NATS-style subjects and queue groups, plus the queue worker runtime.

The worker semantics reproduce internal/queue/nats.go:40-83: decode the Task, sleep until
NotBefore, run the handler, and on error re-publish with Attempts+1 and NotBefore = now +
1s*2^Attempts until MaxAttempts (default 5), then log "task permanently failed". One extension:
an optional ``on_permanent_failure`` hook lets agents mark the document ``failed`` instead of
leaving it ``processing`` forever.

Unlike Core NATS, subjects under ``tasks.`` are buffered while no subscriber exists (the
reference loses them, README.md:717-722).
"""
from __future__ import annotations

import asyncio
import datetime as dt
import itertools
import time
from collections import defaultdict

from ..utils import faults, metrics
from .task import Handler, Task, group_for, next_retry, prepare_for_publish, subject_for


class _Sub:
    def __init__(self, group: str | None):
        self.group = group
        self.q: asyncio.Queue = asyncio.Queue()


class InProcBus:
    def __init__(self, durable_prefix: str = "tasks."):
        self.subs: dict[str, list[_Sub]] = defaultdict(list)
        self.rr: dict[tuple, itertools.count] = {}
        self.pending: dict[str, list[bytes]] = defaultdict(list)
        self.durable_prefix = durable_prefix
        self.published = 0

    def subscribe(self, subject: str, group: str | None = None) -> _Sub:
        s = _Sub(group)
        self.subs[subject].append(s)
        for data in self.pending.pop(subject, []):
            self._deliver(subject, data)
        return s

    def unsubscribe(self, subject: str, sub: _Sub):
        if sub in self.subs.get(subject, []):
            self.subs[subject].remove(sub)

    def publish(self, subject: str, data: bytes):
        self.published += 1
        if not self.subs.get(subject):
            if subject.startswith(self.durable_prefix):
                self.pending[subject].append(data)
            return
        self._deliver(subject, data)

    def _deliver(self, subject: str, data: bytes):
        groups: dict[str, list[_Sub]] = defaultdict(list)
        for s in self.subs[subject]:
            if s.group is None:
                s.q.put_nowait(data)
            else:
                groups[s.group].append(s)
        for g, members in groups.items():
            c = self.rr.setdefault((subject, g), itertools.count())
            members[next(c) % len(members)].q.put_nowait(data)


async def run_task(q, task: Task, handler: Handler, log, on_permanent_failure=None):
    """Handle one decoded task with the reference's NotBefore + retry semantics."""
    if task.not_before is not None:
        delay = (task.not_before - dt.datetime.now(dt.timezone.utc)).total_seconds()
        if delay > 0:
            await asyncio.sleep(delay)
    t0 = time.perf_counter()
    try:
        faults.maybe_fail(f"handler.{task.type}")
        await handler(task)
        metrics.TASKS.labels(task.type, "ok").inc()
        metrics.TASK_ATTEMPTS.labels(task.type).observe(task.attempts + 1)
    except Exception as err:  # noqa: BLE001
        nxt = next_retry(task)
        metrics.TASKS.labels(task.type, "retry" if nxt is not None else "permanent_failure").inc()
        if nxt is not None:
            try:
                await q.enqueue(nxt)
            except Exception as e2:  # noqa: BLE001
                log.error("failed to re-enqueue task after failure", "id", task.id, "type", task.type,
                          "original_err", err, "enqueue_err", e2)
        else:
            log.error("task permanently failed", "id", task.id, "type", task.type, "original_err", err)
            if on_permanent_failure is not None:
                try:
                    await on_permanent_failure(task, err)
                except Exception as e3:  # noqa: BLE001
                    log.error("permanent-failure hook failed", "err", e3)
    finally:
        metrics.TASK_SECONDS.labels(task.type).observe(time.perf_counter() - t0)


class InProcQueue:
    def __init__(self, bus: InProcBus, log, concurrency: int = 1):
        self.bus, self.log, self.concurrency = bus, log, concurrency

    async def enqueue(self, task: Task) -> None:
        faults.maybe_fail("queue.enqueue")
        prepare_for_publish(task)
        self.bus.publish(subject_for(task.type), task.encode())

    async def worker(self, task_type: str, handler: Handler, stop: asyncio.Event | None = None,
                     on_permanent_failure=None) -> None:
        subject = subject_for(task_type)
        sub = self.bus.subscribe(subject, group_for(task_type))
        stop = stop or asyncio.Event()
        sem = asyncio.Semaphore(self.concurrency)
        tasks = set()
        try:
            while not stop.is_set():
                get = asyncio.ensure_future(sub.q.get())
                stopper = asyncio.ensure_future(stop.wait())
                done, _ = await asyncio.wait({get, stopper}, return_when=asyncio.FIRST_COMPLETED)
                if get not in done:
                    get.cancel()
                    stopper.cancel()
                    break
                stopper.cancel()
                data = get.result()
                try:
                    task = Task.decode(data)
                except Exception as e:  # noqa: BLE001
                    self.log.error("failed to decode task", "err", e)
                    continue
                await sem.acquire()

                async def _one(t=task):
                    try:
                        await run_task(self, t, handler, self.log, on_permanent_failure)
                    finally:
                        sem.release()

                fut = asyncio.ensure_future(_one())
                tasks.add(fut)
                fut.add_done_callback(tasks.discard)
        finally:
            self.bus.unsubscribe(subject, sub)
            for t in list(tasks):
                await t
