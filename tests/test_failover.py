"""Replica failure isolation (VERDICT r3 Next #6): a SIGKILLed engine rank fails only the searches
that need its shard; every other replica keeps serving searches, embeds and answers, and the
cluster's health names the dead replica. gloo on CPU, world 4, one process per rank."""
import json
import socket

import torch.multiprocessing as mp

import dist_checks


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_sigkilled_rank_fails_only_its_shard(tmp_path):
    world, port = 4, _port()
    out = str(tmp_path / "failover.json")
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=dist_checks.check_replica_failover, args=(r, world, port, out)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(180)
    alive = [p for p in procs if p.is_alive()]
    for p in alive:
        p.kill()
    assert not alive, "ranks hung"
    assert procs[world - 1].exitcode == -9, [p.exitcode for p in procs]
    assert all(p.exitcode == 0 for p in procs[:world - 1]), [p.exitcode for p in procs]
    v = json.loads(open(out).read())
    print(v)
    assert "error" not in v, v
    assert v["before_all_ok"] and v["live_searches_ok"] and v["embed_search_ok"], v
    assert v["dead_search_failed"] is True, v
    assert v["answers_ok"] and not v["answer_errors"], v
    assert v["health_ok_flag"] is False and v["dead_replicas"] == [world - 1], v
    assert world - 1 in v["shards_down"], v
