"""Tokenizers built locally (there is no network to fetch pretrained vocabularies).

* Encoder: BERT-style WordPiece (lowercase, [CLS]/[SEP]/[PAD]/[UNK]/[MASK]) trained with HF
  ``tokenizers`` on the deterministic synthetic corpus, vocab capped at the encoder's vocab size.
* Decoder: byte-level BPE with the Phi-3 chat special tokens (``<|system|>``, ``<|user|>``,
  ``<|assistant|>``, ``<|end|>``, ``<|endoftext|>``), vocab capped at the decoder's vocab size.

Trained once and cached as JSON under ``DA_CACHE_DIR`` (default ``~/.cache/docagents_amd``);
training is deterministic for a given corpus, so every process and every box gets the same ids.
"""
from __future__ import annotations

import fcntl
import os
from functools import lru_cache
from pathlib import Path

from tokenizers import Tokenizer, decoders, models, normalizers, pre_tokenizers, processors, trainers

from ..text.synthetic import corpus

ENC_SPECIAL = ["[PAD]", "[UNK]", "[CLS]", "[SEP]", "[MASK]"]
DEC_SPECIAL = ["<unk>", "<s>", "<|endoftext|>", "<|system|>", "<|user|>", "<|assistant|>", "<|end|>"]
_VERSION = "v1"


def _cache_dir() -> Path:
    d = Path(os.environ.get("DA_CACHE_DIR", Path.home() / ".cache" / "docagents_amd"))
    d.mkdir(parents=True, exist_ok=True)
    return d


def _locked_build(path: Path, builder):
    lock = path.with_suffix(".lock")
    with open(lock, "w") as lf:
        fcntl.flock(lf, fcntl.LOCK_EX)
        if not path.exists():
            tok = builder()
            tmp = path.with_suffix(".tmp")
            tok.save(str(tmp))
            os.replace(tmp, path)
    return Tokenizer.from_file(str(path))


def _train_encoder(vocab_size: int) -> Tokenizer:
    tok = Tokenizer(models.WordPiece(unk_token="[UNK]", max_input_chars_per_word=100))
    tok.normalizer = normalizers.BertNormalizer(lowercase=True)
    tok.pre_tokenizer = pre_tokenizers.BertPreTokenizer()
    tr = trainers.WordPieceTrainer(vocab_size=vocab_size, special_tokens=ENC_SPECIAL, min_frequency=2)
    tok.train_from_iterator(corpus(1_500_000, seed=11), trainer=tr)
    cls, sep = tok.token_to_id("[CLS]"), tok.token_to_id("[SEP]")
    tok.post_processor = processors.TemplateProcessing(single="[CLS] $A [SEP]", pair="[CLS] $A [SEP] $B [SEP]",
                                                       special_tokens=[("[CLS]", cls), ("[SEP]", sep)])
    tok.decoder = decoders.WordPiece()
    return tok


def _train_decoder(vocab_size: int) -> Tokenizer:
    tok = Tokenizer(models.BPE(unk_token=None, byte_fallback=False))
    tok.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=False)
    tok.decoder = decoders.ByteLevel()
    tr = trainers.BpeTrainer(vocab_size=vocab_size, special_tokens=DEC_SPECIAL, min_frequency=2,
                             initial_alphabet=pre_tokenizers.ByteLevel.alphabet())
    tok.train_from_iterator(corpus(1_500_000, seed=13), trainer=tr)
    return tok


@lru_cache(maxsize=8)
def encoder_tokenizer(vocab_size: int = 30522) -> Tokenizer:
    p = _cache_dir() / f"enc_wordpiece_{vocab_size}_{_VERSION}.json"
    if p.exists():
        return Tokenizer.from_file(str(p))
    return _locked_build(p, lambda: _train_encoder(vocab_size))


@lru_cache(maxsize=8)
def decoder_tokenizer(vocab_size: int = 32064) -> Tokenizer:
    p = _cache_dir() / f"dec_bpe_{vocab_size}_{_VERSION}.json"
    if p.exists():
        return Tokenizer.from_file(str(p))
    return _locked_build(p, lambda: _train_decoder(vocab_size))


class ChatFormat:
    """Phi-3 style chat prompt (system / user / assistant turns)."""

    def __init__(self, tok: Tokenizer):
        self.tok = tok
        self.eos_ids = {tok.token_to_id("<|end|>"), tok.token_to_id("<|endoftext|>")}
        self.eos_ids.discard(None)

    def prompt(self, system: str, user: str) -> str:
        return f"<|system|>\n{system}<|end|>\n<|user|>\n{user}<|end|>\n<|assistant|>\n"

    def encode(self, system: str, user: str) -> list[int]:
        return self.tok.encode(self.prompt(system, user), add_special_tokens=False).ids

    def decode(self, ids: list[int]) -> str:
        return self.tok.decode(ids, skip_special_tokens=True)

    def decode_many(self, seqs: list[list[int]]) -> list[str]:
        return self.tok.decode_batch([list(x) for x in seqs], skip_special_tokens=True) if len(seqs) > 1 \
            else [self.decode(x) for x in seqs]
