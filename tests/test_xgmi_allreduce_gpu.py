"""xGMI IPC all-reduce (ops/csrc/allreduce.hip) on real GPUs: 2 ranks, one process each. On a 1-GPU
box both ranks share the card (the peer mapping is then same-device IPC: it proves the protocol,
counters, parity and graph capture; cross-GPU coherence over xGMI needs a multi-GPU node)."""
import json
import socket

import pytest
import torch.multiprocessing as mp

from docagents_amd.parallel import selftest

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_xgmi_allreduce_matches_rank_order_sum(tmp_path):
    out = tmp_path / "ar.json"
    mp.spawn(selftest.check_xgmi_allreduce, args=(2, _port(), str(out)), nprocs=2, join=True)
    v = json.loads(out.read_text())
    bad = [c for c in v["cases"] if not c["ok"]]
    assert v["ok"] and not bad, bad
    assert v["calls"] >= 15


def test_tp2_decoder_gpu_uses_xgmi_allreduce(tmp_path):
    out = tmp_path / "tp.json"
    mp.spawn(selftest.check_tp_decoder_gpu, args=(2, _port(), str(out)), nprocs=2, join=True)
    v = json.loads(out.read_text())
    assert v["xgmi"] and v["xgmi_calls"] > 0, v
    assert sum(v["first_equal"]) >= 3, v
    assert sum(v["agree"]) / len(v["agree"]) >= 0.6, v
    assert v["max_prob_diff"] < 0.05, v
