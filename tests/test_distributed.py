"""Distributed correctness without a cluster: gloo on CPU, world 2 / 4 / 8 — the
8-rank cases rehearse the node the scaling bench runs on (index shard per GPU, TP=8 decoder)."""
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
    assert v["max_logit_diff"] < 0.05, v  # bf16 rounding only (logits ~1, ulp 0.008)
    assert v["same_tokens"], v
    assert v["max_prob_diff"] < 1e-3


def test_tp8_decoder_one_kv_head_per_rank_matches_unsharded(tmp_path):
    """TP=8 with 8 KV heads (one per rank, as Llama-3-70B at TP=8): identical greedy tokens."""
    v = _run(selftest.check_tp8_decoder, 8, tmp_path)
    assert v["max_logit_diff"] < 0.05, v
    assert v["same_tokens"], v
    assert v["max_prob_diff"] < 1e-3, v


@pytest.mark.parametrize("world", [2, 4, 8])
def test_sharded_index_exact(tmp_path, world):
    assert _run(selftest.check_sharded_index, world, tmp_path)["exact"]


@pytest.mark.parametrize("world", [2, 4])
def test_engine_group_fanout(tmp_path, world):
    v = _run(selftest.check_engine_group, world, tmp_path)
    assert v["embed_ok"] and v["search_ok"] and v["answer_ok"] and v["embed_index_ok"], v
    assert v["owners"] == list(range(world)) and v["ranks"] == world


@pytest.mark.parametrize("world", [2, 8])
def test_ivf_distributed_kmeans(tmp_path, world):
    v = _run(selftest.check_ivf_kmeans, world, tmp_path)
    assert v["centroids_equal"], v
    assert v["recall"] >= 0.8, v
