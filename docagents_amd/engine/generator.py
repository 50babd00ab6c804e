"""Batched generation: packed varlen prefill + HIP-graph-replayed decode steps.

One decode step (32 layers x ~9 kernels + sampler) is captured once per batch bucket into a HIP
graph (``torch.cuda.CUDAGraph`` on ROCm = hipGraph) and replayed; all per-step bookkeeping
(sampled token -> next input, position/length advance, EOS / max-new-token stop, history write,
confidence accumulation) happens inside the sampler kernel, so the host only checks completion
every few steps. The reference's equivalent is one OpenAI chat call per request
(internal/llm/openai.go:40-105).
"""
from __future__ import annotations

import math
import time

import numpy as np
import torch

from ..models.llama import DecodeState, LlamaDecoder, pack_prompts


def _bucket(n: int) -> int:
    b = 1
    while b < n:
        b *= 2
    return b


class GenResult:
    __slots__ = ("tokens", "mean_prob", "n_tokens")

    def __init__(self, tokens, mean_prob, n_tokens):
        self.tokens, self.mean_prob, self.n_tokens = tokens, mean_prob, n_tokens


class Generator:
    def __init__(self, model: LlamaDecoder, max_batch: int = 64, max_seq: int = 4096, temperature: float = 0.2,
                 seed: int = 0, eos=(), use_graphs: bool = True, max_prefill_tokens: int = 32768,
                 check_every: int = 16):
        self.model = model
        self.max_batch = max_batch
        self.temperature, self.seed = temperature, seed
        self.eos = tuple(e for e in eos if e is not None)[:4]
        self.is_cuda = model.device.type == "cuda"
        self.use_graphs = use_graphs and self.is_cuda
        self.max_prefill_tokens = max_prefill_tokens
        self.check_every = check_every
        if model.cache is None:
            # one extra slot: the dummy slot for padded rows of a bucket
            model.alloc_cache(max_batch + 1, max_seq)
        self.cache = model.cache
        self.dummy_slot = self.cache.acquire(1)[0]
        self.states: dict[tuple, DecodeState] = {}
        self.stats = {"prefill_s": 0.0, "decode_s": 0.0, "prefill_tokens": 0, "decode_steps": 0, "decode_tokens": 0,
                      "calls": 0}
        if self.is_cuda:
            from ..ops import kernels
            c = model.cfg
            nsplit = math.ceil(self.cache.max_seq / 256)
            need = max(max_batch * model.hl * nsplit * (c.head_dim + 2) * 4,
                       8 * max_batch * max(c.ffn * 2 // model.tp.size, c.vocab) * 4)
            kernels.reserve_workspace(need, model.device)

    # --------------------------------------------------------------------------------
    def _state(self, B: int, max_new: int) -> DecodeState:
        key = (B, max_new)
        st = self.states.get(key)
        if st is None:
            st = DecodeState(self.model, B, max_new, self.temperature, self.seed, self.eos)
            self.states[key] = st
        return st

    def _capture(self, st: DecodeState):
        # warm up on a side stream (allocator + lazy init), then capture one step
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        saved = [t.clone() for t in (st.tokens, st.pos, st.lens, st.active, st.hist, st.conf)]
        with torch.cuda.stream(s):
            for _ in range(2):
                self.model.decode_step(st)
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self.model.decode_step(st)
        for t, v in zip((st.tokens, st.pos, st.lens, st.active, st.hist, st.conf), saved):
            t.copy_(v)
        st.graph = g

    def _prefill_into(self, st: DecodeState, prompts, slots, row0: int):
        """Prefill prompts (rows row0..) in token-bounded chunks; sample each first token."""
        m, dev = self.model, self.model.device
        i = 0
        n = len(prompts)
        while i < n:
            j, tot = i, 0
            while j < n and (j == i or tot + len(prompts[j]) <= self.max_prefill_tokens):
                tot += len(prompts[j])
                j += 1
            chunk = prompts[i:j]
            flat, pos, cu, lens = pack_prompts(chunk)
            slot_tok = np.repeat(np.asarray(slots[i:j], dtype=np.int32), lens)
            last = (cu[1:] - 1).astype(np.int64)
            t0 = time.perf_counter()
            to = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev, non_blocking=True)  # noqa: E731
            logits = m.prefill(to(flat), to(pos), to(slot_tok), to(cu), int(lens.max()), to(last))
            r0, r1 = row0 + i, row0 + j
            m.ops.sample(logits, self.temperature, self.seed, 0, out_tok=st.tokens[r0:r1], out_lp=st.lp[r0:r1],
                         conf=st.conf[r0:r1], active=st.active[r0:r1], ctr=st.pos[r0:r1], pos=st.pos[r0:r1],
                         lens=st.lens[r0:r1], hist=st.hist[r0:r1], start=st.start[r0:r1], eos=self.eos)
            self.stats["prefill_tokens"] += int(tot)
            self.stats["prefill_s"] += time.perf_counter() - t0
            i = j

    def generate(self, prompts: list[list[int]], max_new: int) -> list[GenResult]:
        out: list[GenResult] = []
        for s in range(0, len(prompts), self.max_batch):
            out.extend(self._generate_wave(prompts[s:s + self.max_batch], max_new))
        return out

    def _generate_wave(self, prompts, max_new: int) -> list[GenResult]:
        m = self.model
        n = len(prompts)
        if n == 0:
            return []
        max_new = max(1, max_new)
        for p in prompts:
            if len(p) + max_new > self.cache.max_seq:
                raise ValueError(f"prompt of {len(p)} tokens + {max_new} new exceeds the context ({self.cache.max_seq})")
            if len(p) == 0:
                raise ValueError("empty prompt")
        B = min(_bucket(n), self.max_batch) if self.use_graphs else n
        st = self._state(B, max_new)
        slots = self.cache.acquire(n)
        try:
            self.stats["calls"] += 1
            plen = np.asarray([len(p) for p in prompts], dtype=np.int32)
            host = np.zeros((5, B), dtype=np.int32)
            host[0, :n] = plen - 1               # pos: last prompt position (sampling ctr)
            host[1, :n] = plen                   # lens (unused by prefill sampling)
            host[2, :n] = slots
            host[2, n:] = self.dummy_slot
            host[3, :n] = 1                      # active
            host[4, :n] = plen - 1               # start
            dev = m.device
            ht = torch.from_numpy(host).to(dev)
            st.pos.copy_(ht[0]); st.lens.copy_(ht[1]); st.slot.copy_(ht[2]); st.active.copy_(ht[3])
            st.start.copy_(ht[4])
            st.tokens.zero_(); st.hist.fill_(-1); st.conf.zero_()
            self._prefill_into(st, prompts, slots, 0)
            # padded rows: keep them inside the dummy slot's first positions
            if B > n:
                st.pos[n:].zero_(); st.lens[n:].fill_(1)
            t0 = time.perf_counter()
            steps = max_new - 1
            if steps > 0:
                if self.use_graphs and st.graph is None:
                    self._capture(st)
                done = 0
                while done < steps:
                    k = min(self.check_every, steps - done)
                    for _ in range(k):
                        if st.graph is not None:
                            st.graph.replay()
                        else:
                            m.decode_step(st)
                        # padded rows never advance past the dummy slot's capacity
                    done += k
                    self.stats["decode_steps"] += k
                    if done < steps and int(st.active[:n].sum().item()) == 0:
                        break
                    if B > n:
                        st.pos[n:].zero_(); st.lens[n:].fill_(1)
            hist = st.hist[:n].cpu().numpy()
            conf = st.conf[:n].cpu().numpy()
            self.stats["decode_s"] += time.perf_counter() - t0
        finally:
            self.cache.release(slots)
        res = []
        for b in range(n):
            toks = [int(t) for t in hist[b] if t >= 0]
            # drop EOS from the text
            toks = [t for t in toks if t not in self.eos]
            cnt = float(conf[b, 1])
            res.append(GenResult(toks, float(conf[b, 0] / cnt) if cnt > 0 else 1.0, int(cnt)))
            self.stats["decode_tokens"] += int(cnt)
        return res
