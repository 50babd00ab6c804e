"""Native C++ runtime: the NATS-protocol broker (queue groups, durable buffering, ack/redelivery,
DLQ) and the RESP key-value cache, driven through the framework's own asyncio clients."""
import asyncio
import os
import socket
import subprocess
import time

import pytest

from docagents_amd.cache.cache import KVCache, QueryResult, Source
from docagents_amd.native import binary
from docagents_amd.queue.broker_client import BrokerClient, BrokerQueue
from docagents_amd.queue.task import Task
from docagents_amd.utils.log import discard


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def wait_port(port, timeout=10):
    t0 = time.time()
    while time.time() - t0 < timeout:
        try:
            socket.create_connection(("127.0.0.1", port), 0.2).close()
            return
        except OSError:
            time.sleep(0.05)
    raise TimeoutError(port)


@pytest.fixture
def broker():
    port = free_port()
    p = subprocess.Popen([str(binary("da-broker")), "--listen", f"127.0.0.1:{port}", "--ack-wait", "1",
                          "--max-deliver", "3"], stderr=subprocess.DEVNULL)
    wait_port(port)
    yield f"nats://127.0.0.1:{port}"
    p.kill()
    p.wait()


@pytest.fixture
def kvserver():
    port = free_port()
    p = subprocess.Popen([str(binary("da-kvserver")), "--listen", f"127.0.0.1:{port}", "--requirepass", "pw"],
                         stderr=subprocess.DEVNULL)
    wait_port(port)
    yield f"127.0.0.1:{port}"
    p.kill()
    p.wait()


def test_broker_pubsub_queue_groups(broker):
    async def go():
        a = await BrokerClient(broker).connect()
        b = await BrokerClient(broker).connect()
        pub = await BrokerClient(broker).connect()
        _, qa = await a.subscribe("tasks.parse", "workers-parse")
        _, qb = await b.subscribe("tasks.parse", "workers-parse")
        _, qall = await a.subscribe("tasks.*")  # plain wildcard subscriber sees everything
        await pub.flush()
        for i in range(20):
            await pub.publish("tasks.parse", str(i).encode())
        await pub.flush()
        await asyncio.sleep(0.2)
        got = []
        for q in (qa, qb):
            while not q.empty():
                got.append(int((await q.get())[1]))
        assert sorted(got) == list(range(20)) and qall.qsize() == 20
        stats = await pub.request("$SYS.REQ.STATS")
        assert b'"subs":4' in stats  # 3 + the request inbox
        for c in (a, b, pub):
            await c.close()
    asyncio.run(go())


def test_broker_durable_buffer_and_redelivery(broker):
    async def go():
        pub = await BrokerClient(broker).connect()
        for i in range(3):  # nobody subscribed yet: buffered
            await pub.publish("tasks.analyze", f"m{i}".encode())
        await pub.flush()
        w1 = await BrokerClient(broker).connect()
        _, q1 = await w1.subscribe("tasks.analyze", "workers-analyze")
        msgs = [await asyncio.wait_for(q1.get(), 2) for _ in range(3)]
        assert sorted(m[1] for m in msgs) == [b"m0", b"m1", b"m2"]
        assert all(m[2].startswith("$ACK.") for m in msgs)
        await w1.publish(msgs[0][2], b"")  # ack only the first
        await w1.flush()
        # worker dies with two unacked messages -> redelivered to the next member
        w2 = await BrokerClient(broker).connect()
        _, q2 = await w2.subscribe("tasks.analyze", "workers-analyze")
        await w2.flush()
        w1.closed = True
        w1.writer.close()
        re = sorted([(await asyncio.wait_for(q2.get(), 3))[1] for _ in range(2)])
        assert re == [b"m1", b"m2"]
        # never acked: redelivered on ack-wait timeout until max-deliver, then dead-lettered
        dlq = await BrokerClient(broker).connect()
        _, qd = await dlq.subscribe("$DLQ.>")
        await dlq.flush()
        got = await asyncio.wait_for(qd.get(), 8)
        assert got[0] == "$DLQ.tasks.analyze"
        for c in (pub, w2, dlq):
            await c.close()
    asyncio.run(go())


def test_broker_queue_worker_end_to_end(broker):
    async def go():
        q = await BrokerQueue(broker, discard()).connect()
        seen = []
        stop = asyncio.Event()

        async def h(t):
            seen.append(t.payload)
            if len(seen) == 5:
                stop.set()
        w = asyncio.ensure_future(q.worker("parse", h, stop))
        await asyncio.sleep(0.1)
        for i in range(5):
            await q.enqueue(Task(type="parse", payload=f"p{i}".encode()))
        await asyncio.wait_for(w, 5)
        assert sorted(seen) == [f"p{i}".encode() for i in range(5)]
        await q.close()
    asyncio.run(go())


def test_kvserver_cache_client(kvserver):
    async def go():
        with pytest.raises(Exception):
            await KVCache(kvserver, "wrong").connect()
        c = await KVCache(kvserver, "pw").connect()
        assert await c.get_query_result("k") is None
        r = QueryResult("ans", 0.5, [Source("c1", 0.8, "p")])
        await c.set_query_result("k", r, 1)
        got = await c.get_query_result("k")
        assert got.answer == "ans" and got.sources[0].chunk_id == "c1"
        await c.set_embedding("what?", [0.25, -0.5], 100)
        assert await c.get_embedding("what?") == [0.25, -0.5]
        raw = await c._cmd("GET", "embed:" + __import__("hashlib").sha256(b"what?").hexdigest())
        assert raw == b"[0.25, -0.5]"
        await asyncio.sleep(1.2)
        assert await c.get_query_result("k") is None  # EX expiry
        await c.set_query_result("k2", r, 100)
        await c.invalidate_document("any")  # reference semantics: drops every query:* key
        assert await c.get_query_result("k2") is None and await c.get_embedding("what?") is not None
        assert await c._cmd("DBSIZE") == 1
        await c.close()
    asyncio.run(go())


def test_kernel_debug_build_compiles(tmp_path):
    """The DA_DEBUG (device-assert) variant of the kernels cross-compiles for gfx950."""
    import shutil
    import subprocess

    import pytest

    from docagents_amd.ops import build as B
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("hipcc not available")
    src = B.CSRC / "rope_sample.hip"
    r = subprocess.run([hipcc, *B._flags(True), "-c", str(src), "-o", str(tmp_path / "dbg.o")],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]


def test_kvserver_client_reconnects_after_server_restart():
    """A KV server restart (same address) costs the client the commands in flight, not the cache:
    the next command after the backoff reconnects (AUTH first) and the cache works again; while the
    server is down, commands fail fast instead of hanging."""
    port = free_port()
    cmd = [str(binary("da-kvserver")), "--listen", f"127.0.0.1:{port}", "--requirepass", "pw"]
    p = subprocess.Popen(cmd, stderr=subprocess.DEVNULL)
    wait_port(port)

    async def go():
        nonlocal p
        c = await KVCache(f"127.0.0.1:{port}", "pw", timeout=2.0).connect()
        c.RECONNECT_S = 0.2
        await c._cmd("SET", "a", "1", "EX", 100)
        p.kill()
        p.wait()
        with pytest.raises(Exception):
            await c._cmd("GET", "a")  # the loss surfaces on the command in flight
        t0 = time.monotonic()
        with pytest.raises(Exception):
            await c._cmd("GET", "a")  # server down: a fast failure
        assert time.monotonic() - t0 < 1.5
        p = subprocess.Popen(cmd, stderr=subprocess.DEVNULL)
        wait_port(port)
        await asyncio.sleep(0.3)  # past the backoff
        assert await c._cmd("GET", "a") is None  # a fresh server: reconnected, authenticated
        await c._cmd("SET", "b", "2", "EX", 100)
        assert await c._cmd("GET", "b") == b"2"
        assert c.reconnects >= 1
        await c.close()
    try:
        asyncio.run(go())
    finally:
        p.kill()
        p.wait()


def test_kvserver_client_pipelines_concurrent_commands(kvserver):
    """The RESP client pipelines: 300 concurrent SET / GET from one connection (replies matched in
    FIFO order), an error reply fails only its own command, and a closed server fails every
    pending command instead of hanging it."""
    async def go():
        c = await KVCache(kvserver, "pw").connect()

        async def one(i):
            await c._cmd("SET", f"pk{i}", f"v{i}", "EX", 100)
            return await c._cmd("GET", f"pk{i}")
        got = await asyncio.gather(*[one(i) for i in range(300)])
        assert got == [f"v{i}".encode() for i in range(300)]
        res = await asyncio.gather(c._cmd("GET", "pk1"), c._cmd("NOSUCHCMD"), c._cmd("GET", "pk2"),
                                   return_exceptions=True)
        assert res[0] == b"v1" and isinstance(res[1], Exception) and res[2] == b"v2", res
        await c.close()
    asyncio.run(go())
