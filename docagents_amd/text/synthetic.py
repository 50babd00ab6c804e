"""Deterministic synthetic corpus: pseudo-English words with a Zipfian distribution.

Used for tokenizer training (no network => no pretrained vocabularies), synthetic documents in
tests/benchmarks and synthetic questions. Everything is a pure function of the seed.
"""
from __future__ import annotations

import random

_ONSETS = ["", "b", "c", "d", "f", "g", "h", "j", "k", "l", "m", "n", "p", "r", "s", "t", "v", "w", "z",
           "br", "cr", "dr", "fl", "gr", "pl", "pr", "sh", "st", "th", "tr", "ch", "sp", "str"]
_VOWELS = ["a", "e", "i", "o", "u", "ai", "ea", "io", "ou", "oo", "ie"]
_CODAS = ["", "", "n", "r", "s", "t", "l", "m", "nd", "st", "ng", "rk", "ck", "x"]
_COMMON = ["the", "of", "and", "to", "in", "a", "is", "that", "for", "it", "as", "with", "was", "on", "be",
           "by", "this", "are", "or", "from", "at", "which", "an", "not", "data", "system", "document",
           "agent", "query", "model", "result", "process", "value", "time", "report"]


def make_lexicon(n: int = 20000, seed: int = 1234) -> list[str]:
    rng = random.Random(seed)
    words = list(_COMMON)
    seen = set(words)
    while len(words) < n:
        syl = rng.choice([1, 2, 2, 3, 3, 4])
        w = "".join(rng.choice(_ONSETS) + rng.choice(_VOWELS) + rng.choice(_CODAS) for _ in range(syl))
        if w and w not in seen:
            seen.add(w)
            words.append(w)
    return words


class TextGen:
    def __init__(self, seed: int = 0, lexicon_size: int = 20000):
        self.lex = make_lexicon(lexicon_size)
        self.rng = random.Random(seed)
        # Zipf weights via cumulative table
        w = [1.0 / (i + 1) ** 1.07 for i in range(len(self.lex))]
        tot = 0.0
        self.cum = []
        for x in w:
            tot += x
            self.cum.append(tot)
        self.total = tot

    def word(self) -> str:
        import bisect
        return self.lex[min(bisect.bisect_left(self.cum, self.rng.random() * self.total), len(self.lex) - 1)]

    def sentence(self, lo: int = 6, hi: int = 18) -> str:
        n = self.rng.randint(lo, hi)
        ws = [self.word() for _ in range(n)]
        ws[0] = ws[0].capitalize()
        s = " ".join(ws)
        if self.rng.random() < 0.15:
            s += ", " + " ".join(self.word() for _ in range(self.rng.randint(2, 6)))
        return s + self.rng.choice([".", ".", ".", "?", "!"])

    def paragraph(self, n_words: int) -> str:
        out, cnt = [], 0
        while cnt < n_words:
            s = self.sentence()
            out.append(s)
            cnt += len(s.split())
        return " ".join(out)

    def document(self, n_words: int) -> str:
        paras, cnt = [], 0
        while cnt < n_words:
            p = self.paragraph(min(120, n_words - cnt + 5))
            paras.append(p)
            cnt += len(p.split())
        return "\n\n".join(paras)

    def question(self, source: str | None = None) -> str:
        if source:
            ws = source.split()
            if len(ws) > 12:
                i = self.rng.randint(0, len(ws) - 10)
                frag = " ".join(ws[i:i + self.rng.randint(5, 9)])
                return f"What does the document say about {frag.rstrip('.?!,')}?"
        return "What is " + " ".join(self.word() for _ in range(self.rng.randint(3, 8))) + "?"


def corpus(n_chars: int = 2_000_000, seed: int = 7) -> list[str]:
    g = TextGen(seed)
    lines, tot = [], 0
    while tot < n_chars:
        p = g.paragraph(80)
        lines.append(p)
        tot += len(p)
    return lines
