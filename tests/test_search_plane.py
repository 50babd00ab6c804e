"""The owner-routed search plane (parallel/search_plane.py) in one process, two ranks over real
sockets: exact merged results, routing only to owner shards, a HUNG shard (accepts, never answers)
failing only the searches that need it (by timeout, naming it), and a restarted shard rejoining
without coordination."""
import socket
import threading
import time

import numpy as np
import pytest
import torch

from docagents_amd.index.flat import FlatIndex
from docagents_amd.parallel.search_plane import SearchPlane, ShardUnavailable, owner_of


def _unit(n, d, seed):
    x = np.random.default_rng(seed).standard_normal((n, d)).astype(np.float32)
    return x / np.linalg.norm(x, axis=1, keepdims=True)


def _docs(world, per, prefix="sp"):
    out, i = {r: [] for r in range(world)}, 0
    while min(len(v) for v in out.values()) < per:
        d = f"{prefix}-{i}"
        i += 1
        r = owner_of(d, world)
        if len(out[r]) < per:
            out[r].append(d)
    return out


def _pair(timeout_s=2.0, retry_s=0.2):
    d = 32
    idx = [FlatIndex(d, "cpu"), FlatIndex(d, "cpu")]
    planes = [SearchPlane(idx[r], r, 2, timeout_s=timeout_s, retry_s=retry_s) for r in range(2)]
    addrs = [p.listen() for p in planes]
    for p in planes:
        p.connect(addrs).start()
    docs = _docs(2, 4)
    X = {}
    for r in range(2):
        for j, doc in enumerate(docs[r]):
            v = _unit(3, d, 100 * r + j)
            X[doc] = v
            idx[r].add(doc, np.arange(3) + 1000 * r + 10 * j, torch.from_numpy(v))
    return planes, idx, docs, X


def _exact(q, docs, X, k):
    rows = [(float(X[dd][i] @ q), dd, i) for dd in docs for i in range(3)]
    return sorted((s for s, _, _ in rows), reverse=True)[:k]


def test_plane_exact_and_routed():
    planes, idx, docs, X = _pair()
    try:
        q = _unit(2, 32, 7)
        flt = [docs[0][:2] + docs[1][:1], docs[0][2:3]]  # row 1 needs only rank 0's shard
        s, keys = planes[1].submit(q, 4, -1.0, flt).result(10)
        for b in range(2):
            got = sorted(s[b][keys[b] >= 0].tolist(), reverse=True)
            assert np.allclose(got, _exact(q[b], flt[b], X, 4), atol=2e-2)
        st = planes[1].stats
        assert st["remote_parts"] == 1 and st["local_parts"] == 1  # one request per owner shard
        s2, k2 = planes[0].submit(q[:1], 3, -1.0, [docs[0]]).result(10)
        assert planes[0].stats["remote_parts"] == 0  # all documents local: no network hop
        assert (k2 >= 0).all()
        # unknown / empty filter: nothing to match, no request sent
        s3, k3 = planes[0].submit(q[:1], 3, -1.0, [[]]).result(10)
        assert (k3 < 0).all()
    finally:
        for p in planes:
            p.stop(timeout=2)


def test_hung_shard_times_out_alone_and_restarted_shard_rejoins():
    planes, idx, docs, X = _pair(timeout_s=1.0, retry_s=0.1)
    q = _unit(1, 32, 9)
    try:
        # rank 1's shard server "hangs": replace it by a socket that accepts and never answers
        addr = planes[0].addrs[1]
        planes[0].peers[1].close()  # the peer process "died": its connections are gone
        planes[1].stop(timeout=2)
        time.sleep(0.2)
        hung = socket.socket()
        hung.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        hung.bind(addr)
        hung.listen(8)
        conns = []
        threading.Thread(target=lambda: conns.append(hung.accept()), daemon=True).start()
        t0 = time.monotonic()
        with pytest.raises(Exception) as ei:
            planes[0].submit(q, 3, -1.0, [docs[0][:1] + docs[1][:1]]).result(10)
        assert "[1]" in str(ei.value) or "shard 1" in str(ei.value), ei.value
        assert time.monotonic() - t0 < 5
        # searches that only need rank 0 are unaffected
        s, k = planes[0].submit(q, 3, -1.0, [docs[0]]).result(10)
        assert (k >= 0).all()
        hung.close()
        for c, _ in conns:
            c.close()
        # rank 1 comes back on the same address: the next request reconnects
        planes[1] = SearchPlane(idx[1], 1, 2, port=addr[1], timeout_s=2.0)
        planes[1].listen()
        planes[1].connect(planes[0].addrs).start()
        time.sleep(0.3)
        deadline = time.monotonic() + 5
        while True:
            try:
                s, k = planes[0].submit(q, 3, -1.0, [docs[1]]).result(10)
                break
            except (ShardUnavailable, TimeoutError):
                assert time.monotonic() < deadline
                time.sleep(0.2)
        assert (k >= 0).all() and planes[0].health()["shards_down"] == []
    finally:
        for p in planes:
            p.stop(timeout=2)


def test_timed_out_parts_leave_no_pending_callbacks():
    planes, idx, docs, X = _pair(timeout_s=0.5, retry_s=0.1)
    try:
        addr = planes[0].addrs[1]
        planes[0].peers[1].close()
        planes[1].stop(timeout=2)
        time.sleep(0.2)
        hung = socket.socket()
        hung.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        hung.bind(addr)
        hung.listen(8)
        conns = []
        threading.Thread(target=lambda: conns.append(hung.accept()), daemon=True).start()
        q = _unit(1, 32, 3)
        for _ in range(3):
            with pytest.raises(TimeoutError):
                planes[0].submit(q, 3, -1.0, [docs[1][:1]]).result(10)
        time.sleep(0.3)
        assert planes[0].peers[1].pending == {} and planes[0].searches == {}
        hung.close()
        for c, _ in conns:
            c.close()
    finally:
        for p in planes:
            p.stop(timeout=2)


def test_requester_that_stops_reading_does_not_stall_the_shard():
    """A client that sends big searches and never reads the replies fills its socket buffers; the
    shard's scan worker must keep serving everyone else (replies leave through a per-connection
    writer thread, not the scan thread)."""
    from docagents_amd.parallel.search_plane import _send_frame
    planes, idx, docs, X = _pair(timeout_s=5.0)
    stuck = socket.create_connection(planes[0].addrs[0])
    stuck.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 4096)
    try:
        big = _unit(512, 32, 11)
        for i in range(8):  # 8 replies of 512 x 1024 (scores + keys) = ~6 MB each, never read
            _send_frame(stuck, {"id": 10_000 + i, "vecs": big, "k": 1024, "thr": -1.0, "filters": None})
        time.sleep(1.0)  # the shard has scanned them and is stuck writing to this client (old design)
        q = _unit(1, 32, 12)
        t0 = time.monotonic()
        s, k = planes[1].submit(q, 3, -1.0, [docs[0][:2]]).result(10)  # a part served by rank 0
        assert (k >= 0).all() and time.monotonic() - t0 < 3
        assert planes[0].stats["served_remote"] >= 9
    finally:
        stuck.close()
        for p in planes:
            p.stop(timeout=2)


def test_shard_that_accepts_but_never_reads_never_blocks_submit():
    """a remote shard that accepts connections but never reads them (a stopped
    process) fills the requester's send buffer. submit() must return at once (the frame goes out on
    the peer's writer thread), the send times out and marks the shard down, the searches that need
    it fail, and searches on other shards keep running meanwhile."""
    d = 32
    idx = FlatIndex(d, "cpu")
    docs = _docs(2, 3)
    for j, doc in enumerate(docs[0]):
        idx.add(doc, np.arange(3) + 10 * j, torch.from_numpy(_unit(3, d, j)))
    mute = socket.socket()
    mute.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 4096)  # accepted sockets inherit it
    mute.bind(("127.0.0.1", 0))
    mute.listen(8)
    held = []
    threading.Thread(target=lambda: held.append(mute.accept()), daemon=True).start()
    plane = SearchPlane(idx, 0, 2, timeout_s=6.0, send_timeout_s=0.5, retry_s=0.1)
    plane.listen()
    plane.connect([plane.listen(), mute.getsockname()]).start()
    try:
        big = _unit(4096, d, 5)  # 512 KB of fp32 per request: the kernel buffers fill quickly
        futs = []
        t0 = time.monotonic()
        for _ in range(6):
            futs.append(plane.submit(big, 3, -1.0, [docs[1][:1]] * len(big)))
        assert time.monotonic() - t0 < 1.0  # never blocked on the mute shard's socket
        s, k = plane.submit(_unit(1, d, 6), 3, -1.0, [docs[0]]).result(5)  # local shard unaffected
        assert (k >= 0).all()
        errs = []
        for f in futs:
            with pytest.raises(Exception) as ei:
                f.result(30)
            errs.append(str(ei.value))
        # the send timeout (buffers full) or the search deadline (frames buffered, never answered)
        assert all("shard 1" in e or "[1]" in e for e in errs), errs[:3]
    finally:
        plane.stop(timeout=2)
        mute.close()
        for c, _ in held:
            c.close()


def test_shard_refuses_parts_past_its_queue_cap_and_drops_expired_ones(monkeypatch):
    """a shard whose scan worker is stalled stops queueing after _QUEUED_ROWS_MAX
    rows (the part fails at once) and drops queued parts whose requester deadline has passed."""
    import docagents_amd.parallel.search_plane as SP
    monkeypatch.setattr(SP, "_QUEUED_ROWS_MAX", 64)
    idx = FlatIndex(32, "cpu")
    plane = SearchPlane(idx, 0, 1, timeout_s=5.0)  # not started: nothing drains the queue
    got = []
    for i in range(3):
        plane._enqueue(SP._Job(_unit(32, 32, i), 3, -1.0, None, lambda s, g: got.append("ok"),
                               lambda e: got.append(repr(e)), deadline=time.monotonic() - 1 if i == 0 else None))
    assert plane.stats["refused"] == 1 and "overloaded" in got[-1]
    take = plane._take()  # the expired part is dropped (failed), the live one is scanned
    assert len(take) == 1 and plane.stats["expired"] == 1 and "expired" in got[-1]
    assert plane._queued_rows == 0


def test_send_backlog_honours_the_search_deadline():
    """a frame that waited in a peer's send backlog past its search's deadline is dropped
    there (never scanned for a requester that gave up), and a frame that is sent carries what is
    LEFT of the deadline as its ttl, not the full timeout."""
    import threading
    import time
    from types import SimpleNamespace

    from docagents_amd.parallel.search_plane import _Peer
    plane = SimpleNamespace(_stop=False, stats={"expired": 0}, retry_s=5.0, connect_timeout_s=0.2, send_timeout_s=0.2)
    srv = socket.socket()
    srv.bind(("127.0.0.1", 0))
    srv.listen(1)
    got = {}
    done = threading.Event()

    def accept():
        c, _ = srv.accept()
        got["conn"] = c
        done.set()
    threading.Thread(target=accept, daemon=True).start()
    peer = _Peer(plane, 1, srv.getsockname())
    fails = []
    peer.send(1, {"id": 1}, lambda *a: None, fails.append, deadline=time.monotonic() - 0.01)
    msg = {"id": 2, "ttl": 30.0}
    peer.send(2, msg, lambda *a: None, fails.append, deadline=time.monotonic() + 10.0)
    assert done.wait(5)
    t0 = time.monotonic()
    while "ttl" in msg and msg["ttl"] == 30.0 and time.monotonic() - t0 < 5:
        time.sleep(0.01)
    assert len(fails) == 1 and isinstance(fails[0], TimeoutError), fails
    assert plane.stats["expired"] == 1
    assert 9.0 < msg["ttl"] <= 10.0  # the remaining time, not the full 30 s
    plane._stop = True
    got["conn"].close()
    srv.close()
