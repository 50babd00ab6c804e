"""SEARCH_TRANSPORT=rccl (parallel/collective_plane.py) rehearsed on the CPU: three gloo ranks, each
owning a shard. Searches submitted on two ranks (different k / floor / filters, one rank idle) come
back equal to the exact single-index search; a stop on one rank ends the rounds on every rank; a
rank that dies fails the others' searches instead of hanging them."""
import os
import socket
import time

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from docagents_amd.config import load
from docagents_amd.index.flat import FlatIndex
from docagents_amd.parallel.search_plane import owner_of

D = 32


def _unit(n, d, seed):
    x = np.random.default_rng(seed).standard_normal((n, d)).astype(np.float32)
    return x / np.linalg.norm(x, axis=1, keepdims=True)


def _corpus(world):
    docs = [f"cp-{i}" for i in range(12)]
    X = {d: _unit(3, D, 50 + i) for i, d in enumerate(docs)}
    ids = {d: np.arange(3) + 100 * i for i, d in enumerate(docs)}
    return docs, X, ids


def _exact(q, flt, X, ids, k, thr):
    rows = [(float(X[d][i] @ q), int(ids[d][i])) for d in flt for i in range(3)]
    rows = [r for r in sorted(rows, key=lambda t: -t[0]) if r[0] >= thr][:k]
    return [s for s, _ in rows], [g for _, g in rows]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _setup(rank, world, port, device="cpu"):
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    import datetime
    ctrl = dist.new_group(backend="gloo", timeout=datetime.timedelta(seconds=5))
    data = dist.new_group(backend="gloo")
    docs, X, ids = _corpus(world)
    idx = FlatIndex(D, device)
    for d in docs:
        if owner_of(d, world) == rank:
            idx.add(d, ids[d], torch.from_numpy(X[d]))
    from docagents_amd.parallel.collective_plane import CollectiveSearchPlane
    plane = CollectiveSearchPlane(idx, rank, world, data, ctrl, device=device, timeout_s=10.0, idle_s=0.002).start()
    return plane, docs, X, ids


def _exact_rank(rank, world, port, device="cpu"):
    plane, docs, X, ids = _setup(rank, world, port, device)
    try:
        if rank == 0:
            q = _unit(3, D, 7)
            flt = [docs[:5], docs[3:9], docs]
            s, g = plane.submit(q, 4, -1.0, flt).result(20)
            for b in range(3):
                es, eg = _exact(q[b], flt[b], X, ids, 4, -1.0)
                assert np.allclose(s[b][:len(es)], es, atol=2e-2), (b, s[b], es)
                assert sorted(g[b][:len(eg)].tolist()) == sorted(eg)
            s2, g2 = plane.submit(q[:1], 2, 0.05, [[]]).result(20)  # filters on nothing
            assert (g2 < 0).all()
        elif rank == 1:
            q = _unit(5, D, 8)
            s, g = plane.submit(q, 6, 0.1, None).result(20)  # no filter: every shard's rows, floor 0.1
            for b in range(5):
                es, eg = _exact(q[b], docs, X, ids, 6, 0.1)
                assert np.allclose(s[b][:len(es)], es, atol=2e-2)
                assert (g[b][len(es):] < 0).all() and (s[b][len(es):] == -np.inf).all()
        # rank 2 (of 3) submits nothing: it still joins every round
        dist.barrier()
        st = plane.stats
        assert st["rounds"] >= 1 and plane.health()["ok"]
        if rank == world - 1:
            plane.stop()
        else:
            t0 = time.monotonic()
            while plane.healthy and time.monotonic() - t0 < 10:
                time.sleep(0.01)
            h = plane.health()
            assert not h["ok"] and plane.stopped_by == world - 1 and sorted(h["shards_down"]) == sorted(
                r for r in range(world) if r != rank)
            with pytest.raises(RuntimeError):
                plane.submit(_unit(1, D, 3), 2, -1.0, None).result(5)
            plane.stop()
    finally:
        dist.destroy_process_group()


def _dead_rank(rank, world, port):
    plane, docs, X, ids = _setup(rank, world, port)
    dist.barrier()
    if rank == 1:
        os._exit(0)  # dies without stopping: its peers' next round fails
    time.sleep(0.5)
    fut = plane.submit(_unit(1, D, 4), 3, -1.0, [docs])
    with pytest.raises(Exception):
        fut.result(15)
    t0 = time.monotonic()
    while plane.healthy and time.monotonic() - t0 < 15:
        time.sleep(0.05)
    assert not plane.health()["ok"] and plane.error
    plane.stop(timeout=2)
    os._exit(0)  # the process group lost a member: skip its teardown


def _scan_fail_rank(rank, world, port):
    plane, docs, X, ids = _setup(rank, world, port)
    try:
        if rank == 1:  # this shard's scans raise for one round only
            real = plane.index.search_ids
            calls = {"n": 0}

            def flaky(*a, **kw):
                calls["n"] += 1
                if calls["n"] == 1:
                    raise RuntimeError("injected scan failure")
                return real(*a, **kw)
            plane.index.search_ids = flaky
        dist.barrier()
        if rank == 0:
            q = _unit(2, D, 11)
            with pytest.raises(RuntimeError, match="failed their scan"):
                plane.submit(q, 3, -1.0, [docs, docs]).result(20)
            s, g = plane.submit(q, 3, -1.0, [docs, docs]).result(20)  # the next round is whole again
            es, eg = _exact(q[0], docs, X, ids, 3, -1.0)
            assert np.allclose(s[0], es, atol=2e-2) and sorted(g[0].tolist()) == sorted(eg)
        dist.barrier()
        assert plane.health()["ok"]  # a failed scan does not end the transport
        if rank == world - 1:
            plane.stop()
        else:
            t0 = time.monotonic()
            while plane.healthy and time.monotonic() - t0 < 10:
                time.sleep(0.01)
            plane.stop()
    finally:
        dist.destroy_process_group()


def _idle_rank(rank, world, port):
    """An idle world backs off: <= 25 control gathers per second per rank; the first search after
    the idle period still completes in < 100 ms (its peers join within idle_max_s = 50 ms)."""
    plane, docs, X, ids = _setup(rank, world, port)
    try:
        dist.barrier()
        time.sleep(0.3)  # past the backoff ramp (2, 4, ..., 50 ms)
        g0, t0 = plane.stats["idle_gathers"], time.monotonic()
        time.sleep(2.0)
        rate = (plane.stats["idle_gathers"] - g0) / (time.monotonic() - t0)
        assert rate <= 25, rate
        if rank == 0:
            t1 = time.perf_counter()
            s, g = plane.submit(_unit(1, D, 9), 3, -1.0, [docs]).result(20)
            ms = (time.perf_counter() - t1) * 1000
            assert ms < 100, ms
            es, eg = _exact(_unit(1, D, 9)[0], docs, X, ids, 3, -1.0)
            assert sorted(g[0].tolist()) == sorted(eg)
        dist.barrier()
        if rank == world - 1:
            plane.stop()
        else:
            t0 = time.monotonic()
            while plane.healthy and time.monotonic() - t0 < 10:
                time.sleep(0.01)
            plane.stop()
    finally:
        dist.destroy_process_group()


def _stop_fails_queued_rank(rank, world, port):
    """A peer's stop fails the searches still QUEUED here (left out of the last round), at once —
    not when their deadline passes."""
    plane, docs, X, ids = _setup(rank, world, port)
    try:
        fut = None
        if rank == 0:
            plane._take = lambda: []  # this rank never takes its work: it stays queued
            fut = plane.submit(_unit(1, D, 5), 3, -1.0, [docs])
        dist.barrier()
        if rank == world - 1:
            time.sleep(0.2)
            plane.stop()
        if rank == 0:
            t0 = time.monotonic()
            with pytest.raises(RuntimeError, match="stopped by rank"):
                fut.result(8)
            assert time.monotonic() - t0 < 5  # well before the 10 s search deadline
            plane.stop()
        elif rank != world - 1:
            plane.stop()
    finally:
        dist.destroy_process_group()


def _local_fail_rank(rank, world, port):
    """A failure in one rank's own post-collective work (the merge) fails that round's searches on
    that rank only; the transport stays up and the next round is exact."""
    from docagents_amd.parallel import collective_plane as CP
    plane, docs, X, ids = _setup(rank, world, port)
    try:
        if rank == 0:
            real = CP.merge_shard_topk
            calls = {"n": 0}

            def flaky(*a, **kw):
                calls["n"] += 1
                if calls["n"] == 1:
                    raise RuntimeError("injected merge failure")
                return real(*a, **kw)
            CP.merge_shard_topk = flaky
        dist.barrier()
        if rank == 0:
            q = _unit(1, D, 13)
            with pytest.raises(RuntimeError, match="injected merge failure"):
                plane.submit(q, 3, -1.0, [docs]).result(20)
            s, g = plane.submit(q, 3, -1.0, [docs]).result(20)
            es, eg = _exact(q[0], docs, X, ids, 3, -1.0)
            assert sorted(g[0].tolist()) == sorted(eg)
            assert plane.stats["local_failures"] == 1
        dist.barrier()
        assert plane.health()["ok"]
        if rank == world - 1:
            plane.stop()
        else:
            t0 = time.monotonic()
            while plane.healthy and time.monotonic() - t0 < 10:
                time.sleep(0.01)
            plane.stop()
    finally:
        dist.destroy_process_group()


def test_collective_plane_idle_backoff_and_wake():
    mp.spawn(_idle_rank, args=(3, _free_port()), nprocs=3, join=True)


def test_collective_plane_peer_stop_fails_queued_searches():
    mp.spawn(_stop_fails_queued_rank, args=(3, _free_port()), nprocs=3, join=True)


def test_collective_plane_local_failure_fails_its_round_only():
    mp.spawn(_local_fail_rank, args=(2, _free_port()), nprocs=2, join=True)


def test_collective_plane_failed_scan_fails_its_round_only():
    mp.spawn(_scan_fail_rank, args=(2, _free_port()), nprocs=2, join=True)


def test_collective_plane_exact_and_coordinated_stop():
    mp.spawn(_exact_rank, args=(3, _free_port()), nprocs=3, join=True)


def test_collective_plane_dead_rank_fails_searches_instead_of_hanging():
    mp.spawn(_dead_rank, args=(2, _free_port()), nprocs=2, join=True)


@pytest.mark.gpu
def test_collective_plane_on_device_ranks():
    """Two ranks on cuda:0 (gloo stages the all-gathers through the host on one GPU; RCCL needs a
    GPU per rank): the rounds' scans, packing and topk_merge on the device, on the round thread's
    own stream and scan workspace, exact vs the single index."""
    mp.spawn(_exact_rank, args=(2, _free_port(), "cuda:0"), nprocs=2, join=True)


def test_search_transport_config():
    assert load({}).validate_engine().search_transport == "plane"
    assert load({"SEARCH_TRANSPORT": "rccl"}).validate_engine().search_transport == "rccl"
    with pytest.raises(ValueError, match="TP_SIZE=1"):
        load({"SEARCH_TRANSPORT": "rccl", "TP_SIZE": "2"}).validate_engine()
    with pytest.raises(ValueError, match="not supported"):
        load({"SEARCH_TRANSPORT": "tcp"}).validate_engine()
