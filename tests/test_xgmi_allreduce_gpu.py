"""xGMI IPC all-reduce (ops/csrc/allreduce.hip) on real GPUs: 2 ranks, one process each. On a 1-GPU
box both ranks share the card (the peer mapping is then same-device IPC: it proves the protocol,
counters, parity and graph capture; cross-GPU coherence over xGMI needs a multi-GPU node)."""
import json
import socket

import pytest
import torch.multiprocessing as mp

import dist_checks

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_xgmi_allreduce_matches_rank_order_sum(tmp_path):
    out = tmp_path / "ar.json"
    mp.spawn(dist_checks.check_xgmi_allreduce, args=(2, _port(), str(out)), nprocs=2, join=True)
    v = json.loads(out.read_text())
    bad = [c for c in v["cases"] if not c["ok"]]
    assert v["ok"] and not bad, bad
    assert v["calls"] >= 15


def test_xgmi_allreduce_rmsnorm_bit_identical_to_unfused(tmp_path):
    """Fused all-reduce + RMSNorm epilogue == all-reduce kernel then rmsnorm kernel, bit for bit."""
    out = tmp_path / "arn.json"
    mp.spawn(dist_checks.check_xgmi_allreduce_norm, args=(2, _port(), str(out)), nprocs=2, join=True)
    v = json.loads(out.read_text())
    bad = [c for c in v["cases"] if not c["ok"]]
    assert v["ok"] and not bad, bad
    assert len(v["cases"]) >= 12


def test_bench_xgmi_cross_device_check_passes(tmp_path):
    """bench.py's multi-GPU C3 check (exact sums one-/two-shot, fused norm bit identity, timing)."""
    out = tmp_path / "vt.json"
    mp.spawn(dist_checks.check_xgmi_verify_and_time, args=(2, _port(), str(out)), nprocs=2, join=True)
    v = json.loads(out.read_text())
    assert v["ok"] and v["fused_norm_bit_identical"] and len(v["cases"]) == 3, v
    assert any(c["twoshot"] for c in v["cases"]), v
    assert set(v["us_per_call"]) == {"16KB", "384KB", "6MB"}, v
    assert all(r["xgmi"] > 0 for r in v["us_per_call"].values()) and v["us_per_call"]["6MB"]["twoshot"], v


def test_xgmi_communicators_recreated_in_one_process(tmp_path):
    """Create / use / close communicators repeatedly (bench.py's N > 1 sequence): exact sums every
    round, and the exported buffers pooled and reused instead of freed (an uncached buffer allocated
    after an exported one was freed could not be exported on an 8-rank rehearsal)."""
    out = tmp_path / "reuse.json"
    mp.spawn(dist_checks.check_xgmi_reuse, args=(2, _port(), str(out)), nprocs=2, join=True)
    v = json.loads(out.read_text())
    assert v["ok"], v
    # three staging sizes (2 x 32 MB, 2 x 512 KB, 2 x 16 MB) and the two signal blocks that were
    # live at once: rounds 2 and 4 reused round 1's buffers, round 3 one signal block
    assert v["pooled_buffers"] == 3 + 2, v


def _tp_ok(v) -> bool:
    return (v["max_logit_diff"] < 0.05 and v["checked"] >= 0.6 * v["decisions"]
            and v["checked_agree"] == v["checked"] and all(v["prefix_ok"]) and v["max_prob_diff"] < 1e-3)


def test_tp2_decoder_gpu_uses_xgmi_allreduce(tmp_path):
    """Per-decision TP verdict (tests/dist_checks.py check_tp_decoder_gpu): teacher-forced logit bound,
    every rounding-proof greedy decision identical, identical tokens up to the first undecidable step."""
    out = tmp_path / "tp.json"
    mp.spawn(dist_checks.check_tp_decoder_gpu, args=(2, _port(), str(out)), nprocs=2, join=True)
    v = json.loads(out.read_text())
    assert v["xgmi"] and v["xgmi_calls"] > 0, v
    assert _tp_ok(v), v


def test_tp2_decoder_gpu_check_bites_on_wrong_shard_order(tmp_path):
    out = tmp_path / "tpw.json"
    mp.spawn(dist_checks.check_tp_decoder_gpu_wrong_order, args=(2, _port(), str(out)), nprocs=2, join=True)
    v = json.loads(out.read_text())
    assert not _tp_ok(v), v
