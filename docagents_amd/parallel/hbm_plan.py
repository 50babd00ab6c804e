"""Per-rank HBM plan of ``bench.py``: what each phase holds on one GPU, from the size formulas the
code allocates with.

The driver runs ``bench.py --gpus N`` at its default arguments on a whole node. Each phase must fit
the 288 GB of one MI355X on its own, and the phases must not stack: the headline's decoder KV cache
(132 slots x 4096 tokens of Phi-3-mini = 213 GB) is released before the N > 1 blocks
(``Engine.release_decoder``), which build their own tensor-parallel decoders and caches.

Every term is the allocation the code makes, by the formula it makes it with:
  decoder weights     ``random_weights`` (embedding whole on every rank, lm_head / layers sharded)
  KV cache            ``KVCache.bytes_for`` (slots x max_seq, kv heads sharded)
  decode workspace    ``Generator.workspace_bytes`` (split-K / split-KV partials)
  prefill transient   one ``max_prefill_tokens`` chunk of activations (x, h, qkv, attention out,
                      gate/up out) — freed between chunks, counted once
  index shard         ``FlatIndex``: rows x (dim bf16 + slot int32 + id int64), built at exactly ``rows``;
                      with ingest the first add grows it 1.5x and the copy holds old + new: +1.5x in
                      the headline, +0.5x after it (config 4 at 1.25M x 1024 peaked 3.3 GB over a
                      plan without the copy)
  index build         ``bench.shard_vectors``: the fp32 draw and its normalised copy, then bf16
                      (setup only: before the first prefill)
  encoder             parameters (+ a second copy for the fp8 / fp16 forms)
  xGMI communicators  2 x (2 x max_bytes staging) + signals per communicator
  runtime             RUNTIME_BYTES for what no formula above sizes: the captured graphs' private
                      pools (decode buckets, encoder buckets), RoPE tables, sampler / prompt buffers,
                      the allocator's block rounding (config 4 fp16 at 1.25M rows measured 0.7 GB
                      over the formula terms)
Reference: the reference sizes nothing (hosted OpenAI / Postgres); docker-compose.yml:84-85,105-106
scales replicas, which is the headline's data-parallel layout here.
"""
from __future__ import annotations

from dataclasses import dataclass

from ..models.configs import DecoderConfig, EncoderConfig, decoder_config, encoder_config

GB = 1e9
HBM_BYTES = 288 * GB
PLAN_LIMIT_BYTES = 270 * GB  # what a phase may hold: the rest is the runtime, RCCL and fragmentation
MAX_PREFILL_TOKENS = 65536   # Generator.max_prefill_tokens default
RUNTIME_BYTES = 2 * GB       # graph pools, tables, small buffers, allocator rounding (every phase)
TP70B_BATCHES = (1, 16)      # tp_decode_70b: decode batches timed
TP70B_WORLD = 8              # tp_decode_70b runs at N = 8 (BASELINE config 5: Llama-3-70B TP=8)


def decoder_weight_bytes(cfg: DecoderConfig, tp: int = 1) -> int:
    """bf16 bytes of one TP rank's decoder weights as ``random_weights`` / ``shard_weights`` lay them
    out: the embedding table whole on every rank, lm_head and every projection split ``tp`` ways."""
    h, d = cfg.hidden, cfg.head_dim
    proj = h * (cfg.heads + 2 * cfg.kv_heads) * d + cfg.heads * d * h + 3 * h * cfg.ffn
    per_layer = proj // tp + 2 * h
    return 2 * (cfg.vocab * h + cfg.vocab * h // tp + cfg.layers * per_layer + h)


def kv_bytes(cfg: DecoderConfig, slots: int, max_seq: int, tp: int = 1) -> int:
    from ..models.llama import KVCache
    return KVCache.bytes_for(cfg, slots, min(max_seq, cfg.max_pos), tp)


def workspace_bytes(cfg: DecoderConfig, max_batch: int, max_seq: int, tp: int = 1) -> int:
    from ..engine.generator import Generator
    return Generator.workspace_bytes(cfg, cfg.heads // tp, tp, max_batch, min(max_seq, cfg.max_pos))


def prefill_transient_bytes(cfg: DecoderConfig, tp: int = 1, tokens: int = MAX_PREFILL_TOKENS) -> int:
    h, d = cfg.hidden, cfg.head_dim
    per_tok = 3 * h + (cfg.heads + 2 * cfg.kv_heads) * d // tp + cfg.heads * d // tp + 2 * cfg.ffn // tp
    return 2 * tokens * per_tok


def encoder_bytes(cfg: EncoderConfig, enc_dtype: str = "bf16") -> int:
    return cfg.param_count() * 2 * (1 if enc_dtype == "bf16" else 2)


def index_bytes(rows: int, dim: int) -> int:
    return rows * (dim * 2 + 4 + 8)


def index_build_bytes(rows: int, dim: int) -> int:
    return rows * dim * (4 + 4 + 2)


def xgmi_bytes(max_bytes: int = 32 << 20, norm_bytes: int = 512 << 10) -> int:
    return 2 * max_bytes + 2 * norm_bytes + (4 << 20)


def round_up(x: int, m: int) -> int:
    return -(-x // m) * m


def tp_decode_max_seq(cfg: DecoderConfig, longest_prompt: int, max_new: int) -> int:
    """``collective_bench.tp_decode``'s cache length: the longest prompt + the decode budget."""
    return min(cfg.max_pos, round_up(longest_prompt + max_new + 8, 256))


@dataclass
class BenchArgs:
    """The ``bench.py`` arguments the plan depends on (defaults = the driver's run)."""
    enc: str = "bge-base"
    llm: str = "phi3-mini"
    batch: int = 128
    max_new: int = 64
    index_rows: int = 100_000
    enc_dtype: str = "bf16"
    tp: int = 1
    overlap: bool = False
    max_seq: int = 4096
    tp70b: bool | None = None  # None: bench.py's "auto" (on at N = 8)
    ingest: bool = True        # --ingest-docs > 0: documents are added to the index (it grows)


def bench_plan(a: BenchArgs, world: int, release_engine_kv: bool = True) -> dict:
    """{phase: {term: bytes, "total": bytes}} for one rank of ``bench.py --gpus world``.
    ``release_engine_kv=False`` models a tree that keeps the headline's KV cache through the N > 1
    blocks (the round-5 bench)."""
    enc, dec = encoder_config(a.enc), decoder_config(a.llm)
    tp = a.tp
    eng_seq = min(a.max_seq, dec.max_pos)
    slots = (2 if a.overlap else 1) * a.batch + 4  # Engine: alloc_cache((2 if overlap) * max_batch + 4)
    resident = {  # held by the engine for the whole run
        "runtime": RUNTIME_BYTES,
        "encoder": encoder_bytes(enc, a.enc_dtype),
        "decoder_weights": decoder_weight_bytes(dec, tp),
        "index": index_bytes(a.index_rows, enc.hidden),
    }
    engine_kv = kv_bytes(dec, slots, eng_seq, tp)
    phases: dict = {}
    setup = dict(resident)
    setup.update({"engine_kv": engine_kv, "index_build": index_build_bytes(a.index_rows, enc.hidden)})
    phases["setup"] = setup
    head = dict(resident)
    head.update({"engine_kv": engine_kv, "workspace": workspace_bytes(dec, a.batch, eng_seq, tp),
                 "prefill_transient": prefill_transient_bytes(dec, tp)})
    if a.ingest:  # FlatIndex._grow at the first add: the 1.5x copy beside the old buffer
        head["index_growth"] = int(1.5 * resident["index"])
    phases["headline"] = head
    kept = dict(resident)
    if a.ingest:
        kept["index_growth"] = int(0.5 * resident["index"])
    if not release_engine_kv:
        kept["engine_kv"] = engine_kv
    kept["workspace"] = head["workspace"]  # the shared workspace only grows
    if world > 1 and tp == 1:
        # tp_decode: the bench decoder at TP = world, cache for maxB + 4 slots; prompts are answer
        # prompts (<= the engine's context budget) -> at most max_seq tokens
        td_seq = tp_decode_max_seq(dec, eng_seq - a.max_new - 8, a.max_new)
        p = dict(kept)
        p.update({"tp_weights": decoder_weight_bytes(dec, world), "tp_kv": kv_bytes(dec, a.batch + 4, td_seq, world),
                  "xgmi": 2 * xgmi_bytes(),
                  "prefill_transient": prefill_transient_bytes(dec, world)})
        p["workspace"] = max(kept["workspace"], workspace_bytes(dec, a.batch, td_seq, world))
        phases["tp_decode"] = p
    if tp == 1 and world > 1 and (a.tp70b if a.tp70b is not None else world == TP70B_WORLD):
        big = decoder_config("llama3-70b")
        td_seq = tp_decode_max_seq(big, eng_seq - a.max_new - 8, a.max_new)
        p = dict(kept)
        p.update({"tp_weights": decoder_weight_bytes(big, world),
                  "tp_kv": kv_bytes(big, max(TP70B_BATCHES) + 4, td_seq, world), "xgmi": 2 * xgmi_bytes(),
                  "prefill_transient": prefill_transient_bytes(big, world)})
        p["workspace"] = max(kept["workspace"], workspace_bytes(big, max(TP70B_BATCHES), td_seq, world))
        phases["tp_decode_70b"] = p
    for p in phases.values():
        p["total"] = sum(v for k, v in p.items() if k != "total")
    return phases


def plan_gb(phases: dict) -> dict:
    return {ph: round(p["total"] / GB, 1) for ph, p in phases.items()}


def check(phases: dict, limit: int = PLAN_LIMIT_BYTES) -> list[str]:
    """Phases over ``limit``: [] when the run fits."""
    return [f"{ph}: {p['total'] / GB:.1f} GB > {limit / GB:.0f} GB" for ph, p in phases.items() if p["total"] > limit]
