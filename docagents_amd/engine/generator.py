"""Batched generation: packed varlen prefill + HIP-graph-replayed decode steps.

One decode step (32 layers x ~9 kernels + sampler) is captured once per batch bucket into a HIP
graph (``torch.cuda.CUDAGraph`` on ROCm = hipGraph) and replayed; all per-step bookkeeping
(sampled token -> next input, position/length advance, EOS / max-new-token stop, history write,
confidence accumulation) happens inside the sampler kernel, so the host only checks completion
every few steps. The reference's equivalent is one OpenAI chat call per request
(internal/llm/openai.go:40-105).
"""
from __future__ import annotations

import collections
import math
import threading
import time
from types import SimpleNamespace

import numpy as np
import torch

from ..models.llama import DecodeState, LlamaDecoder, pack_prompts
from ..ops import h2d


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
                 seed: int = 0, eos=(), use_graphs: bool = True, max_prefill_tokens: int = 65536,
                 check_every: int = 16, share_prefix: bool = True, min_shared_prefix: int = 64):
        self.model = model
        # prompts of one wave that start with the same tokens (the Answer / Summarize system prompt:
        # ~260 tokens of every QA prompt) prefill that head once; see _generate_wave
        self.share_prefix, self.min_shared_prefix = share_prefix, min_shared_prefix
        self.max_batch = max_batch
        self.temperature, self.seed = temperature, seed
        self.eos = tuple(e for e in eos if e is not None)[:4]
        self.is_cuda = model.device.type == "cuda"
        self.use_graphs = use_graphs and self.is_cuda
        # 64k-token chunks: fewer partial tile rounds per GEMM than 32k (same box, 2 rounds each:
        # QA prefill 1103 vs 1119 ms, profiles/r2/ab_prefill_chunk/)
        self.max_prefill_tokens = max_prefill_tokens
        self.check_every = check_every
        if model.cache is None:
            # one extra slot: the dummy slot for padded rows of a bucket
            model.alloc_cache(max_batch + 1, max_seq)
        self.cache = model.cache
        self.dummy_slot = self.cache.acquire(1)[0]
        self.head = None  # {"tokens", "P", "slot"}: the last wave's shared prompt head, kept in its own slot
        self.states: dict[tuple, DecodeState] = {}
        self.stats = {"prefill_s": 0.0, "decode_s": 0.0, "prefill_tokens": 0, "decode_steps": 0, "decode_tokens": 0,
                      "calls": 0, "shared_prefix_tokens": 0}
        # phase timing: synchronize the device around prefill / decode so prefill_s / decode_s are
        # device time (bench breakdown pass); off in serving (a sync per phase costs overlap)
        self.sync_phases = False
        if self.is_cuda:
            from ..ops import kernels
            kernels.reserve_workspace(self.workspace_bytes(model.cfg, model.hl, model.tp.size, max_batch,
                                                           self.cache.max_seq), model.device)

    @staticmethod
    def workspace_bytes(cfg, heads_local: int, tp: int, max_batch: int, max_seq: int) -> int:
        """The shared split-KV / split-K workspace a generator reserves (parallel/hbm_plan.py)."""
        nsplit = math.ceil(max_seq / 256)
        return max(max_batch * heads_local * nsplit * (cfg.head_dim + 2) * 4,
                   8 * max_batch * max(cfg.ffn * 2 // tp, cfg.vocab) * 4)

    def close(self):
        """Give this generator's KV slots (the padded rows' dummy slot, a kept prompt-head slot) back
        to the model's cache and drop its decode states and graphs: several generators may take
        turns on one model's cache (bench.py's TP decode arms)."""
        held = [self.dummy_slot] + ([self._head_slot] if getattr(self, "_head_slot", None) is not None else [])
        self.cache.release(held)
        self._head_slot, self.head, self.dummy_slot = None, None, None
        self.states.clear()

    # --------------------------------------------------------------------------------
    def _persistent_head_slot(self, held: int):
        """The KV slot that keeps the last wave's shared prompt head. Taken once, and only when it
        is a true spare: once this call's ``held`` slots are back, a full wave of max_batch prompts
        must still find its slots (a head slot taken from a cache sized max_batch + 1 would make
        the next full wave fail with 'KV cache exhausted'). None when there is no spare slot."""
        if self.head is not None:
            return self.head["slot"]
        if getattr(self, "_head_slot", None) is None:
            if len(self.cache.free) + held <= self.max_batch:
                return None
            self._head_slot = self.cache.acquire(1)[0]
        return self._head_slot

    def _state(self, B: int, max_new: int, lane: int = 0) -> DecodeState:
        key = (B, max_new, lane)
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

    def shared_prefix_len(self, prompts) -> int:
        """Tokens every prompt of the wave starts with, rounded down to a multiple of 64 (the decode
        attention's key tile), or 0 when sharing does not pay (fewer than 2 prompts or a head
        shorter than min_shared_prefix); at least one token of each prompt stays in its own
        prefill, which produces that prompt's first-token logits."""
        if not self.share_prefix or len(prompts) < 2:
            return 0
        first = prompts[0]
        n = min(len(p) for p in prompts) - 1
        if n < self.min_shared_prefix:
            return 0
        for p in prompts[1:]:
            if p[:n] != first[:n]:
                k = 0
                while k < n and p[k] == first[k]:
                    k += 1
                n = k
                if n < self.min_shared_prefix:
                    return 0
        n -= n % 64
        return n if n >= self.min_shared_prefix else 0

    def _prefill_into(self, st: DecodeState, prompts, slots, row0: int, prefix: tuple[int, int] | None = None):
        """Prefill prompts (rows row0..) in token-bounded chunks; sample each first token.
        prefix = (slot, P): the prompts are suffixes of a P-token head already in ``slot``."""
        m, dev = self.model, self.model.device
        P = 0 if prefix is None else prefix[1]
        i = 0
        n = len(prompts)
        while i < n:
            j, tot = i, 0
            while j < n and (j == i or tot + len(prompts[j]) <= self.max_prefill_tokens):
                tot += len(prompts[j])
                j += 1
            chunk = prompts[i:j]
            flat, pos, cu, lens = pack_prompts(chunk)
            if P:
                pos += P
            slot_tok = np.repeat(np.asarray(slots[i:j], dtype=np.int32), lens)
            last = (cu[1:] - 1).astype(np.int64)
            t0 = time.perf_counter()
            to = lambda a: h2d(a, dev)  # noqa: E731
            logits = m.prefill(to(flat), to(pos), to(slot_tok), to(cu), int(lens.max()), to(last), prefix=prefix,
                               local_logits=True)
            r0, r1 = row0 + i, row0 + j
            m.sample(logits, self.temperature, self.seed, 0, out_tok=st.tokens[r0:r1], out_lp=st.lp[r0:r1],
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
        if not prompts:
            return []
        w = self._wave_begin(prompts, max_new)
        try:
            self._wave_decode(w)
        except BaseException:
            self.cache.release(w.slots)
            raise
        return self._wave_end(w)

    def _wave_begin(self, prompts, max_new: int, lane: int = 0, head_build: bool = True) -> "_Wave":
        """Set up the decode state of one wave (bucketed to B rows) and prefill it on the current
        stream. lane: which of the generator's decode states of that bucket to use (two waves in
        flight need two). head_build=False: never (re)build the shared prompt head (another wave
        may be decoding against the kept head's slot) — a miss then prefills whole prompts."""
        m = self.model
        n = len(prompts)
        max_new = max(1, max_new)
        for p in prompts:
            if len(p) + max_new > self.cache.max_seq:
                raise ValueError(f"prompt of {len(p)} tokens + {max_new} new exceeds the context ({self.cache.max_seq})")
            if len(p) == 0:
                raise ValueError("empty prompt")
        B = min(_bucket(n), self.max_batch) if self.use_graphs else n
        st = self._state(B, max_new, lane)
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
            ht = h2d(host, dev)
            st.pos.copy_(ht[0]); st.lens.copy_(ht[1]); st.slot.copy_(ht[2]); st.active.copy_(ht[3])
            st.start.copy_(ht[4])
            st.tokens.zero_(); st.hist.fill_(-1); st.conf.zero_()
            if self.sync_phases and self.is_cuda:
                torch.cuda.synchronize(dev)
            t_pf = time.perf_counter()
            h = self.head if self.share_prefix else None
            if h is not None and all(len(p) > h["P"] and p[:h["P"]] == h["tokens"] for p in prompts):
                # prompt-head cache hit (a batch-1 query after earlier batches): no head prefill
                P, hslot = h["P"], h["slot"]
                self.stats["head_cache_hits"] = self.stats.get("head_cache_hits", 0) + n
                self.stats["shared_prefix_tokens"] += P * n
            else:
                P = self.shared_prefix_len(prompts) if head_build else 0
                hslot = None
            if P and hslot is None:
                # the shared head once, then only the suffixes, attending to the head's keys in its
                # slot; decode reads keys [0, P) of every row from that slot too (st.pre), so the
                # head's K/V exist once: prefilled once, read from L2/MALL by all rows. The head goes
                # into a slot of its own when one is free and is kept for later calls (a batch-1
                # query then skips it); otherwise into row 0's slot for this call only.
                hslot = self._persistent_head_slot(held=n)
                keep = hslot is not None
                if not keep:
                    hslot = slots[0]
                t0 = time.perf_counter()
                to = lambda a: h2d(a, dev)  # noqa: E731
                m.prefill(to(np.asarray(prompts[0][:P], dtype=np.int32)), to(np.arange(P, dtype=np.int32)),
                          to(np.full(P, hslot, dtype=np.int32)), to(np.array([0, P], dtype=np.int32)), P,
                          to(np.array([P - 1], dtype=np.int64)))
                self.stats["prefill_tokens"] += P
                self.stats["shared_prefix_tokens"] += P * (n - 1)
                self.stats["prefill_s"] += time.perf_counter() - t0
                if keep:
                    self.head = {"tokens": list(prompts[0][:P]), "P": P, "slot": hslot}
            if P:
                self._prefill_into(st, [p[P:] for p in prompts], slots, 0, prefix=(hslot, P))
                pre = np.zeros((B, 2), dtype=np.int32)
                pre[:n] = (P, hslot)
                st.pre.copy_(h2d(pre, dev))
            else:
                st.pre.zero_()
                self._prefill_into(st, prompts, slots, 0)
            # padded rows: keep them inside the dummy slot's first positions
            if B > n:
                st.pos[n:].zero_(); st.lens[n:].fill_(1)
            if self.sync_phases:
                if self.is_cuda:
                    torch.cuda.synchronize(dev)
                self.stats["prefill_wall_s"] = self.stats.get("prefill_wall_s", 0.0) + time.perf_counter() - t_pf
        except BaseException:
            self.cache.release(slots)
            raise
        return _Wave(st, n, B, slots, max_new - 1)

    def _wave_decode(self, w: "_Wave"):
        """The wave's decode steps on the current stream (graph replays; the host checks every
        check_every steps whether every row has stopped)."""
        m, st, n, B = self.model, w.st, w.n, w.B
        w.t0 = time.perf_counter()  # decode_s runs to the results on the host (_wave_end)
        steps = w.steps
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

    def _wave_end(self, w: "_Wave") -> list[GenResult]:
        try:
            hist = w.st.hist[:w.n].cpu().numpy()
            conf = w.st.conf[:w.n].cpu().numpy()
            if w.t0 is not None:
                self.stats["decode_s"] += time.perf_counter() - w.t0
        finally:
            self.cache.release(w.slots)
        res = []
        for b in range(w.n):
            toks = [int(t) for t in hist[b] if t >= 0]
            # drop EOS from the text
            toks = [t for t in toks if t not in self.eos]
            cnt = float(conf[b, 1])
            res.append(GenResult(toks, float(conf[b, 0] / cnt) if cnt > 0 else 1.0, int(cnt)))
            self.stats["decode_tokens"] += int(cnt)
        return res

    def generate_overlapped(self, next_prompts, max_new: int, lanes) -> list[list[GenResult]]:
        """Waves of prompts with the decode of wave i running BESIDE the prefill of wave i + 1.

        The decode of a wave is HBM-bound (KV-cache stream), the prefill MFMA-bound; plain
        concurrent streams interleave them badly (profiles/r1 stream_overlap_probe), and a fixed CU
        partition leaves the prefill on part of the chip after the decode ends
        (profiles/r3/cumask_probe.jsonl). Here: the decode replays on the decode lane (a CU-masked
        stream, ``lanes[0]``) from a helper thread; the next wave's prefill starts on the
        complementary lane (``lanes[1]``) and, before each layer, moves to the full chip as soon as
        the decode has finished (host check, at most two layers issued ahead). Tokens are identical
        to ``generate`` wave by wave (same kernels, same sampler counters).

        next_prompts(i) -> prompts of wave i, or None after the last; it runs on the host while the
        previous wave decodes (its own kernels — question embeds, searches — go to the full chip).
        Returns one result list per wave."""
        dec_s, pf_s = lanes
        full = torch.cuda.current_stream()
        out: list[list[GenResult]] = []
        prompts = next_prompts(0)
        if not prompts:
            return out
        cur = self._wave_begin(prompts, max_new, lane=0)
        try:
            return self._overlap_loop(cur, next_prompts, max_new, dec_s, pf_s, full, out)
        finally:
            self.model.layer_hook = None

    def _overlap_loop(self, cur, next_prompts, max_new, dec_s, pf_s, full, out):
        from ..ops import kernels as K
        i = 1
        while cur is not None:
            if self.use_graphs and cur.st.graph is None and cur.steps > 0:
                self._capture(cur.st)  # never capture while another thread issues work
            dec_s.wait_stream(torch.cuda.current_stream())
            done = torch.cuda.Event()
            recorded = threading.Event()  # an event never recorded reads as complete: gate on this
            err: list = []

            def run_decode(w=cur):
                try:
                    with torch.cuda.stream(dec_s):
                        self._wave_decode(w)
                        done.record(dec_s)
                except BaseException as e:  # noqa: BLE001 - re-raised on the caller's thread
                    err.append(e)
                    done.record(dec_s)
                finally:
                    recorded.set()
            th = threading.Thread(target=run_decode, name="wave-decode", daemon=True)
            t_w = time.perf_counter()
            th.start()
            nxt = None
            failed = None
            try:
                prompts = next_prompts(i)
                if prompts:
                    issued: list = []
                    state = {"moved": False}

                    def hook(li):
                        if state["moved"]:
                            return
                        if len(issued) >= 2:
                            issued[-2].synchronize()
                        if recorded.is_set() and done.query():
                            full.wait_stream(pf_s)
                            torch.cuda.set_stream(full)
                            state["moved"] = True
                            self.stats.setdefault("overlap_moves", []).append((li, round(time.perf_counter() - t_w, 4)))
                            return
                        ev = torch.cuda.Event()
                        ev.record(pf_s)
                        issued.append(ev)
                    pf_s.wait_stream(full)
                    self.model.layer_hook = hook
                    try:
                        with torch.cuda.stream(pf_s), K.workspace_role("prefill"):
                            nxt = self._wave_begin(prompts, max_new, lane=i % 2, head_build=False)
                            end = torch.cuda.current_stream()
                    finally:
                        self.model.layer_hook = None
                    full.wait_stream(end)
            except BaseException as e:  # noqa: BLE001 - the decode thread is joined first
                failed = e
            finally:
                th.join()
            self.stats.setdefault("overlap_decode_join_s", []).append(round(time.perf_counter() - t_w, 4))
            full.wait_stream(dec_s)
            if err or failed is not None:
                torch.cuda.synchronize()
                self.cache.release(cur.slots)
                if nxt is not None:
                    self.cache.release(nxt.slots)
                raise err[0] if err else failed
            out.append(self._wave_end(cur))
            cur = nxt
            i += 1
        return out


class _Wave:
    __slots__ = ("st", "n", "B", "slots", "steps", "t0")

    def __init__(self, st, n, B, slots, steps):
        self.st, self.n, self.B, self.slots, self.steps = st, n, B, slots, steps
        self.t0 = None


class ContinuousScheduler:
    """Continuous batching over one HIP-graph-captured decode bucket of ``B`` rows.

    Requests are admitted into free rows between decode chunks (prefill of the new prompts runs
    as one packed varlen batch, then their rows join the running graph), and a row is reaped and
    reused as soon as its sequence hits EOS or its token budget — so a short answer never waits
    for the longest one in its batch, and requests arriving mid-generation do not wait for the
    whole batch to drain (SURVEY.md §2.5 "continuous batching for the decoder"; the reference
    makes one blocking OpenAI call per request, internal/llm/openai.go:64-105).

    Per-row token budgets share one history buffer of ``max_new_cap`` columns: a row with budget m
    starts writing at column cap - m (``start`` shifted back), so the sampler's "history full"
    stop fires after exactly m tokens with no kernel change. Free rows point at the generator's
    dummy KV slot and stay inactive (the sampler never advances them).

    Not thread-safe: ``submit`` and ``tick`` are called from the engine's single GPU thread.
    """

    def __init__(self, gen: "Generator", B: int | None = None, max_new_cap: int = 256, chunk_steps: int = 8,
                 max_admit_tokens: int | None = None, max_heads: int = 2):
        self.gen, self.m = gen, gen.model
        # Prompt-head cache (automatic prefix caching): a head shared by the prompts of one admission
        # (the Answer system prompt) is prefilled once into a slot of its own and kept; later prompts
        # starting with it prefill only their suffix, and their decode reads the head's keys from
        # that slot (DecodeState.pre). Entries: {"tokens", "P", "slot", "refs", "used"}; LRU among
        # unreferenced entries when a new head needs a slot.
        self.heads: list[dict] = []
        self.max_heads = max_heads if gen.share_prefix else 0
        self.B = B or gen.max_batch
        self.cap = max(1, max_new_cap)
        self.chunk_steps = chunk_steps
        # prompt tokens admitted per tick (prefilled in max_prefill_tokens chunks): a burst of long
        # prompts (a batch of summaries) joins in one or two ticks instead of trickling in at one
        # prefill chunk per tick, which would stretch the decode of the last-admitted rows
        self.max_admit_tokens = max_admit_tokens or 131072  # 4 x 32k-token chunks (deploy-stack tuning)
        self.st = DecodeState(self.m, self.B, self.cap, gen.temperature, gen.seed, gen.eos)
        # row buckets (powers of two up to B): a tick replays the graph of the smallest bucket that
        # holds every occupied row — an unloaded request decodes at batch-1 cost (the GEMV path), not
        # in the full B-row graph. Admission fills the lowest free rows, so occupancy stays compact.
        self.buckets: dict[int, DecodeState] = {self.B: self.st}
        self.rows: list = [None] * self.B        # row -> (tag, slot, budget)
        self.left: list = [None] * self.B        # row -> decode steps it may still need (budget - 1 - steps run)
        self.pending: collections.deque = collections.deque()
        self._reset_rows(list(range(self.B)))
        self.stats = {"admitted": 0, "finished": 0, "ticks": 0, "steps": 0, "head_hits": 0, "heads_built": 0}

    # -------------------------------------------------------------------------------- public
    def submit(self, prompt: list[int], max_new: int, tag=None):
        max_new = max(1, min(int(max_new), self.cap))
        if not prompt:
            raise ValueError("empty prompt")
        if len(prompt) + max_new > self.gen.cache.max_seq:
            raise ValueError(f"prompt of {len(prompt)} tokens + {max_new} new exceeds the context "
                             f"({self.gen.cache.max_seq})")
        self.pending.append((list(prompt), max_new, tag))

    def busy(self) -> bool:
        return bool(self.pending) or any(r is not None for r in self.rows)

    @property
    def n_active(self) -> int:
        return sum(r is not None for r in self.rows)

    def steps_to_free(self) -> int:
        """Decode steps until the first running row reaches its token budget (1 when none runs)."""
        left = [x for x in self.left if x is not None]
        return max(1, min(left)) if left else 1

    def tick(self, steps: int | None = None, stop=None) -> list:
        """Admit what fits, run up to ``steps`` decode steps, return [(tag, GenResult)] of finished
        rows. The steps are capped by the largest remaining token budget of the running rows (no
        replays after every row is done), and ``stop()`` (checked between steps, host-side, no
        device sync) ends the tick early — the server passes "new requests are waiting" so an
        arrival waits for at most one step while an unloaded request runs many steps per tick."""
        self.stats["ticks"] += 1
        done = self._admit()
        if self.n_active:
            st, k = self._bucket_state(), steps or self.chunk_steps
            k = max(1, min(k, max(left for left in self.left if left is not None)))
            if self.gen.use_graphs and st.graph is None:
                self.gen._capture(st)
            t0 = time.perf_counter()
            ran = 0
            # graph replays are asynchronous: without a bound the host would queue all k steps before
            # stop() is ever consulted. With a stop callback at most 2 steps run ahead of the host
            # (an event per step), so an arrival waits ~2 steps, and the GPU never idles.
            ahead: collections.deque = collections.deque()
            track = stop is not None and k > 1 and st.graph is not None
            while ran < k:
                if st.graph is not None:
                    st.graph.replay()
                else:
                    self.m.decode_step(st)
                ran += 1
                if stop is not None and ran < k:
                    if track:
                        ev = torch.cuda.Event()
                        ev.record()
                        ahead.append(ev)
                        if len(ahead) > 2:
                            ahead.popleft().synchronize()
                    if stop():
                        break
            for r, left in enumerate(self.left):
                if left is not None:
                    self.left[r] = max(0, left - ran)
            self.stats["steps"] += ran
            sb = self.stats.setdefault("steps_by_bucket", {})
            sb[st.B] = sb.get(st.B, 0) + ran
            self.gen.stats["decode_steps"] += ran
            done += self._reap()
            self.gen.stats["decode_s"] += time.perf_counter() - t0
        return done

    def run_all(self, prompts, max_new: int) -> list["GenResult"]:
        """Convenience: submit everything and tick until drained (results in submission order)."""
        for i, p in enumerate(prompts):
            self.submit(p, max_new, i)
        out: dict = {}
        while self.busy():
            for tag, r in self.tick():
                out[tag] = r
        return [out[i] for i in range(len(prompts))]

    def warmup(self):
        """Capture every bucket's decode graph now (serving startup), not on a request's path."""
        if not self.gen.use_graphs:
            return
        b = 1
        while b <= self.B:
            st = self._state_for(b)
            if st.graph is None:
                self.gen._capture(st)
            b *= 2

    # -------------------------------------------------------------------------------- internals
    def _state_for(self, b: int) -> DecodeState:
        st = self.buckets.get(b)
        if st is None:
            st = self.buckets[b] = self.st.rows(b)
        return st

    def _bucket_state(self) -> DecodeState:
        top = max(i for i, r in enumerate(self.rows) if r is not None) + 1
        b = _bucket(top) if top < self.B else self.B
        return self._state_for(min(b, self.B))

    def _reset_rows(self, rows):
        if not rows:
            return
        st, dev = self.st, self.m.device
        idx = torch.as_tensor(rows, dtype=torch.long, device=dev)
        st.slot.index_fill_(0, idx, self.gen.dummy_slot)
        st.pos.index_fill_(0, idx, 0)
        st.lens.index_fill_(0, idx, 1)
        st.active.index_fill_(0, idx, 0)
        st.start.index_fill_(0, idx, 0)
        st.pre.index_fill_(0, idx, 0)

    def _match_head(self, prompt):
        for h in self.heads:
            if len(prompt) > h["P"] and prompt[:h["P"]] == h["tokens"]:
                return h
        return None

    def _build_head(self, prompts):
        """Cache the head shared by ``prompts`` (>= 2 of them, >= min_shared_prefix tokens) in a
        slot of its own; None when there is no such head or no slot to spare."""
        P = self.gen.shared_prefix_len(prompts)
        if not P:
            return None
        cache = self.gen.cache
        if len(self.heads) >= self.max_heads:
            idle = [h for h in self.heads if h["refs"] == 0]
            if not idle:
                return None
            old = min(idle, key=lambda h: h["used"])
            self.heads.remove(old)
            cache.release([old["slot"]])
        if not cache.free:
            return None
        slot = cache.acquire(1)[0]
        head = list(prompts[0][:P])
        dev = self.m.device
        to = lambda a: h2d(a, dev)  # noqa: E731
        t0 = time.perf_counter()
        self.m.prefill(to(np.asarray(head, dtype=np.int32)), to(np.arange(P, dtype=np.int32)),
                       to(np.full(P, slot, dtype=np.int32)), to(np.array([0, P], dtype=np.int32)), P,
                       to(np.array([P - 1], dtype=np.int64)))
        self.gen.stats["prefill_tokens"] += P
        self.gen.stats["prefill_s"] += time.perf_counter() - t0
        h = {"tokens": head, "P": P, "slot": slot, "refs": 0, "used": self.stats["ticks"]}
        self.heads.append(h)
        self.stats["heads_built"] += 1
        return h

    def _admit(self) -> list:
        free = [i for i, r in enumerate(self.rows) if r is None]
        take, tot = [], 0
        while self.pending and len(take) < len(free):
            p = self.pending[0]
            if take and tot + len(p[0]) > self.max_admit_tokens:
                break
            take.append(self.pending.popleft())
            tot += len(p[0])
        if not take:
            return []
        # prompt heads: reuse a cached one, or cache the head this admission's prompts share
        hs = [self._match_head(t[0]) for t in take] if self.max_heads else [None] * len(take)
        if self.max_heads:
            miss = [t[0] for t, h in zip(take, hs) if h is None]
            if len(miss) >= 2:
                h = self._build_head(miss)
                if h is not None:
                    hs = [hh if hh is not None else (h if self._match_head(t[0]) is h else None)
                          for t, hh in zip(take, hs)]
        # rows using the same head are prefilled together (suffixes only), plain prompts last
        order = sorted(range(len(take)), key=lambda i: (hs[i] is None, id(hs[i])))
        take, hs = [take[i] for i in order], [hs[i] for i in order]
        n, rows = len(take), free[:len(take)]
        slots = self.gen.cache.acquire(n)
        prompts = [t[0] for t in take]
        plen = np.asarray([len(p) for p in prompts], dtype=np.int32)
        budget = np.asarray([t[1] for t in take], dtype=np.int32)
        dev, i32 = self.m.device, dict(dtype=torch.int32, device=self.m.device)
        tmp = SimpleNamespace(
            tokens=torch.zeros(n, **i32), lp=torch.zeros(n, dtype=torch.float32, device=dev),
            conf=torch.zeros(n, 2, dtype=torch.float32, device=dev), active=torch.ones(n, **i32),
            pos=h2d(plen - 1, dev), lens=h2d(plen.copy(), dev),
            hist=torch.full((n, self.cap), -1, **i32),
            start=h2d(plen - 1 - (self.cap - budget), dev),
            slot=torch.as_tensor(slots, dtype=torch.int32, device=dev))
        i = 0
        pre = np.zeros((n, 2), dtype=np.int32)
        while i < n:
            h, j = hs[i], i
            while j < n and hs[j] is h:
                j += 1
            if h is None:
                self.gen._prefill_into(tmp, prompts[i:j], slots[i:j], i)
            else:
                self.gen._prefill_into(tmp, [p[h["P"]:] for p in prompts[i:j]], slots[i:j], i, prefix=(h["slot"], h["P"]))
                pre[i:j] = (h["P"], h["slot"])
                h["refs"] += j - i
                h["used"] = self.stats["ticks"]
                self.stats["head_hits"] += j - i
                self.gen.stats["shared_prefix_tokens"] += h["P"] * (j - i)
            i = j
        st = self.st
        idx = torch.as_tensor(rows, dtype=torch.long, device=dev)
        for name in ("tokens", "lp", "conf", "active", "pos", "lens", "hist", "start", "slot"):
            getattr(st, name).index_copy_(0, idx, getattr(tmp, name))
        st.pre.index_copy_(0, idx, h2d(pre, dev))
        for r, (p, b, tag), sl, h in zip(rows, take, slots, hs):
            self.rows[r] = (tag, sl, int(b), h)
            self.left[r] = int(b) - 1  # the first token came from the prefill
        self.stats["admitted"] += n
        # a budget of one token (or an immediate EOS) finishes at prefill
        return self._reap(rows)

    def _reap(self, rows=None) -> list:
        rows = [i for i, r in enumerate(self.rows) if r is not None] if rows is None else rows
        if not rows:
            return []
        st = self.st
        act = st.active.cpu().numpy()
        fin = [r for r in rows if self.rows[r] is not None and act[r] == 0]
        if not fin:
            return []
        idx = torch.as_tensor(fin, dtype=torch.long, device=self.m.device)
        hist = st.hist.index_select(0, idx).cpu().numpy()
        conf = st.conf.index_select(0, idx).cpu().numpy()
        out, slots = [], []
        eos = set(self.gen.eos)
        for k, r in enumerate(fin):
            tag, sl, b, h = self.rows[r]
            if h is not None:
                h["refs"] -= 1
            toks = [int(t) for t in hist[k, self.cap - b:] if t >= 0 and int(t) not in eos]
            cnt = float(conf[k, 1])
            out.append((tag, GenResult(toks, float(conf[k, 0] / cnt) if cnt > 0 else 1.0, int(cnt))))
            self.gen.stats["decode_tokens"] += int(cnt)
            self.rows[r] = None
            self.left[r] = None
            slots.append(sl)
        self._reset_rows(fin)
        st.hist.index_fill_(0, idx, -1)
        st.conf.index_fill_(0, idx, 0.0)
        self.gen.cache.release(slots)
        self.stats["finished"] += len(fin)
        return out
