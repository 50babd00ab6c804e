"""The engine entrypoint as deployed on a node (services/engine_main.py under torch.distributed.run):
world 4 on CPU (gloo), TP_SIZE 1 and 2. The agents' client (EngineCluster) connects to the base
URL only, discovers the replicas, routes ingest to the owner's replica, load-balances the rest;
searches span every rank's shard through the search plane; SIGTERM checkpoints every shard and the
restarted engine serves the same rows."""
import asyncio
import os
import signal
import socket
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port_block(n: int) -> int:
    for _ in range(50):
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        base = s.getsockname()[1]
        s.close()
        ok = True
        for p in range(base, base + n):
            t = socket.socket()
            try:
                t.bind(("127.0.0.1", p))
            except OSError:
                ok = False
            finally:
                t.close()
        if ok and base + n < 65000:
            return base
    raise RuntimeError("no free port block")


def _start(tmp_path, base, world, tp, transport="plane"):
    env = dict(os.environ, EMBED_ARCH="tiny-enc", LLM_ARCH="tiny-dec-tp8", TP_SIZE=str(tp), ENGINE_CONTINUOUS="1",
               SEARCH_TRANSPORT=transport,
               INDEX_DIR=str(tmp_path / "index"), INDEX_CHECKPOINT_S="0", ENGINE_LIVENESS_INTERVAL="0",
               DATA_DIR=str(tmp_path), CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", PYTHONPATH=ROOT,
               OMP_NUM_THREADS="1", ENGINE_MAX_BATCH="4", MAX_NEW_TOKENS="4", SUMMARY_MAX_NEW_TOKENS="4")
    log = open(tmp_path / f"engine_{tp}.log", "ab")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", "--master-port", str(base + 20), "-m", "docagents_amd.services", "engine",
           "--listen", f"tcp://127.0.0.1:{base}"]
    return subprocess.Popen(cmd, env=env, stdout=log, stderr=subprocess.STDOUT, cwd=ROOT, start_new_session=True)


def _stop(p):
    if p.poll() is None:
        os.killpg(p.pid, signal.SIGTERM)
        try:
            p.wait(60)
        except subprocess.TimeoutExpired:
            os.killpg(p.pid, signal.SIGKILL)
            p.wait(10)


@pytest.mark.parametrize("tp,transport", [(1, "plane"), (2, "plane"), (1, "rccl")])
def test_engine_main_replicas_route_balance_search_and_recover(tmp_path, tp, transport):
    """transport "rccl": the searches travel in the lock-step collective rounds
    (parallel/collective_plane.py; gloo on these CPU ranks) instead of point to point."""
    from docagents_amd.engine.rpc import EngineCluster
    from docagents_amd.engine.server import owner_of
    world = 4
    base = _port_block(24)
    docs, per, i = [], {}, 0
    while len(docs) < 12:  # three documents on every rank's shard
        d = f"doc-{i}"
        i += 1
        if per.get(owner_of(d, world), 0) < 3:
            docs.append(d)
            per[owner_of(d, world)] = per.get(owner_of(d, world), 0) + 1

    async def phase1():
        cl = await EngineCluster(f"tcp://127.0.0.1:{base}").connect(retries=400, delay=0.25)
        assert cl.replicas == world // tp and cl.topology["world"] == world and cl.topology["tp"] == tp
        res = await asyncio.gather(*[cl.call("embed_index", doc_id=d, keys=np.arange(2, dtype=np.int64) + 10 * i,
                                             texts=[f"{d} part {j} text" for j in range(2)])
                                     for i, d in enumerate(docs)])
        assert [r["rows"] for r in res] == [2] * len(docs)
        rows = await cl.call("index_docs")
        assert rows == {d: 2 for d in docs}
        assert {owner_of(d, world) for d in docs} == set(range(world))
        q = (await cl.call("embed", texts=["doc-3 part 1 text"], preprocess=True))["vecs"]
        s = await cl.call("search", vecs=q, filters=[docs], k=3, min_sim=-1.0)
        assert (np.asarray(s["keys"]) >= 0).all()
        h = await cl.call("health")
        assert h["ok"] and not h.get("shards_down")
        ans = await asyncio.gather(*[cl.call("answer", items=[{"question": f"q{i}?", "context": "ctx",
                                                              "quality": 1.0}]) for i in range(2 * cl.replicas)])
        assert all(len(a["results"]) == 1 for a in ans)
        st = await cl.call("stats")
        assert len(st["replicas"]) == cl.replicas
        planes = [r["search_plane"] for rep in st["replicas"] for r in rep["ranks"]]
        if transport == "rccl":  # every rank joined the rounds that carried the search
            assert len(planes) == world and all(p["transport"] == "gloo" and p["rounds"] >= 1 for p in planes)
        else:
            assert all("transport" not in p for p in planes)
        await cl.close()
        return q, s

    p = _start(tmp_path, base, world, tp, transport)
    try:
        q, before = asyncio.run(phase1())
    finally:
        _stop(p)
    p = _start(tmp_path, base, world, tp, transport)

    async def phase2():
        cl = await EngineCluster(f"tcp://127.0.0.1:{base}").connect(retries=400, delay=0.25)
        rows = await cl.call("index_docs")
        after = await cl.call("search", vecs=q, filters=[docs], k=3, min_sim=-1.0)
        await cl.close()
        return rows, after

    try:
        rows, after = asyncio.run(phase2())
    finally:
        _stop(p)
    assert rows == {d: 2 for d in docs}
    np.testing.assert_array_equal(before["keys"], after["keys"])
    np.testing.assert_allclose(before["scores"], after["scores"], atol=1e-6)


class _FakeReplica:
    """An EngineClient stand-in: ``behaviour(method)`` returns a value or raises."""

    def __init__(self, behaviour):
        self.behaviour, self.calls = behaviour, []

    async def call(self, method, trace="", **args):
        self.calls.append(method)
        return self.behaviour(method)


def _cluster(*replicas):
    from docagents_amd.engine.rpc import EngineCluster
    cl = EngineCluster("tcp://127.0.0.1:1")
    cl.clients = list(replicas)
    cl.inflight = [0] * len(replicas)
    cl.dead_until = [0.0] * len(replicas)
    cl.topology = {"replicas": len(replicas), "tp": 1, "world": len(replicas)}
    return cl


def test_slow_but_alive_replica_is_not_marked_dead_and_generations_are_not_retried():
    """a client-side timeout on a busy replica must not mark it dead for
    dead_s or re-run a generation on another replica (nothing cancels the first one server-side).
    Cheap calls (embed / search) may be re-asked of another replica; a connection failure still
    fails over."""
    import asyncio

    def slow(method):
        raise asyncio.TimeoutError()
    fast = _FakeReplica(lambda m: f"ok-{m}")
    busy = _FakeReplica(slow)

    async def go():
        cl = _cluster(busy, fast)
        with pytest.raises(asyncio.TimeoutError):
            cl._rr = 0
            await cl.call("answer", question="q", context="c", quality=1.0)
        assert fast.calls == [] and cl.dead_until == [0.0, 0.0]   # not retried, nobody marked dead
        cl._rr = 0
        assert await cl.call("embed", texts=["x"]) == "ok-embed"   # cheap: re-asked elsewhere
        assert cl.dead_until == [0.0, 0.0] and fast.calls == ["embed"]

        def gone(method):
            raise ConnectionRefusedError("down")
        dead = _FakeReplica(gone)
        cl2 = _cluster(dead, fast)
        cl2._rr = 0
        assert await cl2.call("answer", question="q", context="c", quality=1.0) == "ok-answer"
        assert cl2.dead_until[0] > 0  # a real failure: skipped for dead_s
    asyncio.run(go())
