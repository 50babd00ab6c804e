"""Per-rank HBM plan of the driver's ``bench.py --gpus N`` run (VERDICT r5 Next #1): every phase of
the default run must fit one MI355X at N = 1, 2, 4, 8. The plan is computed from the size formulas
the code allocates with (KVCache.bytes_for, Generator.workspace_bytes, random_weights' layout), and
its negative control — the round-5 bench, which kept the headline's 213 GB KV cache through the N > 1
blocks — must fail at N = 2."""
import pytest
import torch

from docagents_amd.models.configs import decoder_config
from docagents_amd.models.llama import KVCache, random_weights
from docagents_amd.parallel import hbm_plan as HP

GB = 1e9


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_default_bench_fits_every_world(world):
    phases = HP.bench_plan(HP.BenchArgs(), world)
    assert HP.check(phases) == [], HP.plan_gb(phases)
    want = {"setup", "headline"} | ({"tp_decode"} if world > 1 else set()) | ({"tp_decode_70b"} if world == 8 else set())
    assert set(phases) == want


def test_plan_bites_when_engine_kv_is_kept():
    """The round-5 layout (engine KV cache alive beside tp_decode's TP = 2 decoder) is over 270 GB."""
    bad = HP.check(HP.bench_plan(HP.BenchArgs(), 2, release_engine_kv=False))
    assert bad and bad[0].startswith("tp_decode"), bad


def test_headline_kv_is_the_213_gb_cache():
    p = HP.bench_plan(HP.BenchArgs(), 1)["headline"]
    assert 212e9 < p["engine_kv"] < 213.5e9  # 132 slots x 4096 tokens x 393 KB
    assert p["engine_kv"] == KVCache.bytes_for(decoder_config("phi3-mini"), 132, 4096)


def test_70b_shard_is_a_twentieth_of_hbm():
    p = HP.bench_plan(HP.BenchArgs(), 8)["tp_decode_70b"]
    assert 19e9 < p["tp_weights"] < 20e9 and p["tp_kv"] < 5e9


@pytest.mark.parametrize("arch,tp", [("tiny-dec", 1), ("tiny-dec", 2), ("tiny-dec-tp8", 8)])
def test_weight_formula_matches_allocation(arch, tp):
    """decoder_weight_bytes is what random_weights allocates for one TP rank."""
    cfg = decoder_config(arch)
    w = random_weights(cfg, "cpu", 0, tp_rank=tp - 1, tp_size=tp)
    n = sum(t.numel() * t.element_size() for k, t in w.items() if k != "layers")
    n += sum(t.numel() * t.element_size() for L in w["layers"] for t in L.values())
    assert n == HP.decoder_weight_bytes(cfg, tp)


def test_kv_formula_matches_allocation():
    cfg = decoder_config("tiny-dec")
    c = KVCache(cfg, 5, 256, 2, "cpu")
    assert c.buf.numel() * c.buf.element_size() == HP.kv_bytes(cfg, 5, 256, 2)
    assert c.buf.dtype == torch.bfloat16


def test_setup_phase_counts_the_index_build():
    """The config-4 rehearsal's per-rank peak (34.0 GB, profiles/r6/rehearsal_config4_*) came from
    building a 1.25M x 1024 shard (fp32 draw + normalised copy), not from the QA step."""
    a = HP.BenchArgs(enc="bge-large", enc_dtype="fp16", batch=4, index_rows=1_250_000, max_new=8, tp70b=False,
                     ingest=False)
    p = HP.bench_plan(a, 8)
    assert "tp_decode_70b" not in p
    assert p["setup"]["total"] >= 34.0e9 > p["headline"]["total"]


def test_index_growth_and_runtime_cover_the_measured_config4_peak():
    """BASELINE config 4 on one GPU (BGE-large fp16, 1.25M x 1024 shard, with ingest) measured a
    233.8 GB headline peak (profiles/r6/configs/bench_config4_bge_large_fp16_1p25m_r6_head.json): the plan counts the shard's
    growth copy at the first ingest and the runtime slack, so it bounds that peak; without ingest
    the shard never grows."""
    a = HP.BenchArgs(enc="bge-large", enc_dtype="fp16", index_rows=1_250_000)
    p = HP.bench_plan(a, 1)["headline"]
    assert p["total"] >= 233.8e9 and p["index_growth"] == int(1.5 * p["index"])
    assert HP.check(HP.bench_plan(a, 1)) == []
    q = HP.bench_plan(HP.BenchArgs(enc="bge-large", enc_dtype="fp16", index_rows=1_250_000, ingest=False), 1)
    assert "index_growth" not in q["headline"]
