"""Model architectures (random-init weights of these shapes; no network for checkpoints).

Encoders (BGE / E5 class, BERT layers) replace OpenAI text-embedding-3-* (SURVEY.md §2.4 N1/N2);
decoders (Phi-3-mini / Llama-3) replace gpt-4o-mini for Summarize / Answer (N6/N7).
"""
from __future__ import annotations

from dataclasses import dataclass


@dataclass(frozen=True)
class EncoderConfig:
    name: str
    vocab: int = 30522
    hidden: int = 768
    layers: int = 12
    heads: int = 12
    ffn: int = 3072
    max_pos: int = 512
    type_vocab: int = 2
    eps: float = 1e-12
    pooling: str = "cls"  # "cls" (BGE) or "mean" (E5)

    @property
    def head_dim(self) -> int:
        return self.hidden // self.heads

    def param_count(self) -> int:
        h, f = self.hidden, self.ffn
        per = 4 * h * h + 2 * h * f + 9 * h + f
        return self.vocab * h + self.max_pos * h + self.type_vocab * h + 2 * h + self.layers * per


@dataclass(frozen=True)
class DecoderConfig:
    name: str
    vocab: int
    hidden: int
    layers: int
    heads: int
    kv_heads: int
    ffn: int
    max_pos: int
    rope_theta: float
    eps: float = 1e-5
    tie_embeddings: bool = False

    @property
    def head_dim(self) -> int:
        return self.hidden // self.heads

    def param_count(self) -> int:
        h, d = self.hidden, self.head_dim
        attn = h * (self.heads + 2 * self.kv_heads) * d + self.heads * d * h
        mlp = 3 * h * self.ffn
        emb = self.vocab * h * (1 if self.tie_embeddings else 2)
        return emb + self.layers * (attn + mlp + 2 * h) + h

    def kv_bytes_per_token(self, dtype_bytes: int = 2) -> int:
        return self.layers * 2 * self.kv_heads * self.head_dim * dtype_bytes


ENCODERS = {
    "bge-small": EncoderConfig("bge-small", hidden=384, layers=12, heads=12, ffn=1536),
    "bge-base": EncoderConfig("bge-base"),
    "bge-large": EncoderConfig("bge-large", hidden=1024, layers=24, heads=16, ffn=4096),
    "e5-base": EncoderConfig("e5-base", pooling="mean"),
    "e5-large": EncoderConfig("e5-large", hidden=1024, layers=24, heads=16, ffn=4096, pooling="mean"),
    "tiny-enc": EncoderConfig("tiny-enc", vocab=30522, hidden=128, layers=2, heads=2, ffn=256, max_pos=512),
}

DECODERS = {
    "phi3-mini": DecoderConfig("phi3-mini", vocab=32064, hidden=3072, layers=32, heads=32, kv_heads=32,
                               ffn=8192, max_pos=4096, rope_theta=10000.0),
    "llama3-8b": DecoderConfig("llama3-8b", vocab=128256, hidden=4096, layers=32, heads=32, kv_heads=8,
                               ffn=14336, max_pos=8192, rope_theta=500000.0),
    "llama3-70b": DecoderConfig("llama3-70b", vocab=128256, hidden=8192, layers=80, heads=64, kv_heads=8,
                                ffn=28672, max_pos=8192, rope_theta=500000.0),
    "tiny-dec": DecoderConfig("tiny-dec", vocab=32064, hidden=256, layers=2, heads=4, kv_heads=2, ffn=512,
                              max_pos=4096, rope_theta=10000.0),
    # Llama-3-70B's TP=8 layout in miniature: 8 KV heads (one per rank), GQA group 2, FFN / vocab
    # divisible by 8 ranks (distributed tests, bench.py's TP verdict from 3 ranks); head dim 64, one
    # the GPU decode-attention kernels take
    "tiny-dec-tp8": DecoderConfig("tiny-dec-tp8", vocab=32064, hidden=1024, layers=2, heads=16, kv_heads=8,
                                  ffn=1024, max_pos=4096, rope_theta=500000.0),
}

ALIASES = {"text-embedding-3-large": "bge-large", "text-embedding-3-small": "bge-base",
           "gpt-4o-mini": "phi3-mini"}


def encoder_config(name: str) -> EncoderConfig:
    name = ALIASES.get(name, name)
    if name not in ENCODERS:
        raise ValueError(f"unknown encoder arch {name!r}; choose from {sorted(ENCODERS)}")
    return ENCODERS[name]


def decoder_config(name: str) -> DecoderConfig:
    name = ALIASES.get(name, name)
    if name not in DECODERS:
        raise ValueError(f"unknown decoder arch {name!r}; choose from {sorted(DECODERS)}")
    return DECODERS[name]
