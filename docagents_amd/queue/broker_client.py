"""asyncio client for the NATS core protocol (our native broker, or a real nats-server).

``BrokerQueue`` implements the Queue contract on top of it exactly like the reference's
``natsQueue`` (internal/queue/nats.go): publish to ``tasks.<type>``, queue-subscribe with group
``workers-<type>``, NotBefore sleep + in-band retry via re-publish. When the broker attaches an
``$ACK.<n>`` reply subject (our broker's at-least-once extension) the worker acks after the
handler finished (success, or the retry was re-published), so a crashed worker's task is
redelivered instead of lost. Connection loss -> reconnect with backoff and resubscribe.
"""
from __future__ import annotations

import asyncio
import itertools
import json

from ..utils import faults
from .inproc import run_task
from .task import Handler, Task, group_for, prepare_for_publish, subject_for


class BrokerError(RuntimeError):
    pass


class BrokerClient:
    def __init__(self, url: str, name: str = "docagents", log=None):
        u = url
        for pre in ("nats://", "tcp://", "broker://"):
            if u.startswith(pre):
                u = u[len(pre):]
        host, _, port = u.rpartition(":")
        self.host, self.port = host or "127.0.0.1", int(port or 4222)
        self.name, self.log = name, log
        self.reader = self.writer = None
        self.subs: dict[str, tuple[str, str | None, asyncio.Queue]] = {}
        self.sids = itertools.count(1)
        self.wlock = asyncio.Lock()
        self.pong_waiters: list[asyncio.Future] = []
        self.reader_task = None
        self.closed = False
        self.connected = asyncio.Event()
        self.info = {}

    async def connect(self, timeout: float = 5.0):
        self.reader, self.writer = await asyncio.wait_for(asyncio.open_connection(self.host, self.port), timeout)
        line = await asyncio.wait_for(self.reader.readline(), timeout)
        if line.startswith(b"INFO"):
            try:
                self.info = json.loads(line[5:])
            except ValueError:
                self.info = {}
        opts = {"verbose": False, "pedantic": False, "name": self.name, "lang": "python", "version": "0.1.0",
                "protocol": 1}
        self.writer.write(b"CONNECT " + json.dumps(opts).encode() + b"\r\n")
        for sid, (subj, q, _) in self.subs.items():  # resubscribe after reconnect
            self.writer.write(f"SUB {subj} {q + ' ' if q else ''}{sid}\r\n".encode())
        await self.writer.drain()
        self.reader_task = asyncio.ensure_future(self._read_loop())
        await self.flush(timeout)
        self.connected.set()
        return self

    async def flush(self, timeout: float = 5.0):
        fut = asyncio.get_running_loop().create_future()
        self.pong_waiters.append(fut)
        await self._write(b"PING\r\n")
        await asyncio.wait_for(fut, timeout)

    async def _write(self, data: bytes):
        if self.writer is None:
            raise BrokerError("not connected")
        async with self.wlock:
            self.writer.write(data)
            await self.writer.drain()

    async def publish(self, subject: str, data: bytes, reply: str = ""):
        hdr = f"PUB {subject} {reply + ' ' if reply else ''}{len(data)}\r\n".encode()
        await self._write(hdr + data + b"\r\n")

    async def subscribe(self, subject: str, queue: str | None = None) -> tuple[str, asyncio.Queue]:
        sid = str(next(self.sids))
        q: asyncio.Queue = asyncio.Queue()
        self.subs[sid] = (subject, queue, q)
        await self._write(f"SUB {subject} {queue + ' ' if queue else ''}{sid}\r\n".encode())
        return sid, q

    async def unsubscribe(self, sid: str):
        self.subs.pop(sid, None)
        try:
            await self._write(f"UNSUB {sid}\r\n".encode())
        except Exception:  # noqa: BLE001
            pass

    async def request(self, subject: str, data: bytes = b"", timeout: float = 5.0) -> bytes:
        inbox = f"_INBOX.{self.name}.{next(self.sids)}"
        sid, q = await self.subscribe(inbox)
        try:
            await self.publish(subject, data, inbox)
            _, payload, _ = await asyncio.wait_for(q.get(), timeout)
            return payload
        finally:
            await self.unsubscribe(sid)

    async def _read_loop(self):
        r = self.reader
        try:
            while True:
                line = await r.readline()
                if not line:
                    raise ConnectionError("broker closed the connection")
                if line.startswith(b"MSG"):
                    parts = line.decode().split()
                    subj, sid = parts[1], parts[2]
                    reply = parts[3] if len(parts) == 5 else ""
                    n = int(parts[-1])
                    payload = (await r.readexactly(n + 2))[:-2]
                    s = self.subs.get(sid)
                    if s is not None:
                        s[2].put_nowait((subj, payload, reply))
                elif line.startswith(b"PING"):
                    await self._write(b"PONG\r\n")
                elif line.startswith(b"PONG"):
                    if self.pong_waiters:
                        f = self.pong_waiters.pop(0)
                        if not f.done():
                            f.set_result(True)
                elif line.startswith(b"-ERR"):
                    if self.log:
                        self.log.error("broker error", "err", line.decode().strip())
        except (asyncio.IncompleteReadError, ConnectionError, OSError) as e:
            self.connected.clear()
            if not self.closed:
                asyncio.ensure_future(self._reconnect(e))

    async def _reconnect(self, err):
        delay = 0.1
        while not self.closed:
            try:
                if self.log:
                    self.log.warn("broker connection lost; reconnecting", "err", err)
                await self.connect()
                return
            except Exception as e:  # noqa: BLE001
                err = e
                await asyncio.sleep(delay)
                delay = min(delay * 2, 2.0)

    async def close(self):
        self.closed = True
        if self.reader_task:
            self.reader_task.cancel()
        if self.writer:
            self.writer.close()
            try:
                await self.writer.wait_closed()
            except Exception:  # noqa: BLE001
                pass


class BrokerQueue:
    def __init__(self, url: str, log, concurrency: int = 1):
        self.client = BrokerClient(url, log=log)
        self.log, self.concurrency = log, concurrency

    async def connect(self):
        await self.client.connect()
        return self

    async def enqueue(self, task: Task) -> None:
        faults.maybe_fail("queue.enqueue")
        prepare_for_publish(task)
        if not self.client.connected.is_set():
            await asyncio.wait_for(self.client.connected.wait(), 5.0)
        await self.client.publish(subject_for(task.type), task.encode())

    async def worker(self, task_type: str, handler: Handler, stop: asyncio.Event | None = None,
                     on_permanent_failure=None) -> None:
        sid, q = await self.client.subscribe(subject_for(task_type), group_for(task_type))
        stop = stop or asyncio.Event()
        sem = asyncio.Semaphore(self.concurrency)
        running = set()
        try:
            while not stop.is_set():
                get = asyncio.ensure_future(q.get())
                st = asyncio.ensure_future(stop.wait())
                done, _ = await asyncio.wait({get, st}, return_when=asyncio.FIRST_COMPLETED)
                st.cancel()
                if get not in done:
                    get.cancel()
                    break
                _, data, reply = get.result()
                try:
                    task = Task.decode(data)
                except Exception as e:  # noqa: BLE001
                    self.log.error("failed to decode task", "err", e)
                    if reply.startswith("$ACK."):
                        await self.client.publish(reply, b"")
                    continue
                await sem.acquire()

                async def one(t=task, rep=reply):
                    try:
                        await run_task(self, t, handler, self.log, on_permanent_failure)
                        if rep.startswith("$ACK."):
                            await self.client.publish(rep, b"")
                    finally:
                        sem.release()

                fut = asyncio.ensure_future(one())
                running.add(fut)
                fut.add_done_callback(running.discard)
        finally:
            await self.client.unsubscribe(sid)
            for f in list(running):
                await f

    async def close(self):
        await self.client.close()
