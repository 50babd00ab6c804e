"""Distributed correctness without a cluster: gloo on CPU, world 2/4."""
import json
import socket

import pytest
import torch.multiprocessing as mp

from docagents_amd.parallel import selftest


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(fn, world, tmp_path):
    out = tmp_path / f"{fn.__name__}_{world}.json"
    mp.spawn(fn, args=(world, _port(), str(out)), nprocs=world, join=True)
    return json.loads(out.read_text())


def test_tp2_decoder_matches_unsharded(tmp_path):
    v = _run(selftest.check_tp_decoder, 2, tmp_path)
    assert v["same_tokens"], v
    assert v["max_prob_diff"] < 1e-3


@pytest.mark.parametrize("world", [2, 4])
def test_sharded_index_exact(tmp_path, world):
    assert _run(selftest.check_sharded_index, world, tmp_path)["exact"]


def test_engine_group_fanout(tmp_path):
    v = _run(selftest.check_engine_group, 2, tmp_path)
    assert v["embed_ok"] and v["search_ok"] and v["answer_ok"], v
    assert v["owners"] == [0, 1] and v["ranks"] == 2


def test_ivf_distributed_kmeans(tmp_path):
    v = _run(selftest.check_ivf_kmeans, 2, tmp_path)
    assert v["centroids_equal"], v
    assert v["recall"] >= 0.8, v
