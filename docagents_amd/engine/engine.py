"""The per-GPU inference engine: encoder + decoder + vector index shard.

Implements the reference's outsourced compute contracts on-node:
  * ``Embedder.Embed / EmbedBatch`` (internal/embeddings/embeddings.go:7-10, openai.go:38-127)
    -> ``embed`` (preprocess identically, keep a 1:1 text->vector mapping, unit-norm output);
  * ``llm.Client.Summarize`` (internal/llm/openai.go:40-62) -> ``summarize_many`` with map-reduce over
    the decoder context and the same ``extractSummary`` parsing;
  * ``llm.Client.Answer`` (openai.go:64-105) -> ``answer_many``: confidence = context quality x mean
    token probability of the generated tokens (openai.go:101-102,149-164);
  * ``Store.TopK``'s vector part (internal/store/postgres.go:218-285) -> ``index`` (flat / IVFFlat).
Batching is across requests: texts are packed by tokens, prompts are generated together.
"""
from __future__ import annotations

import threading
import time

import numpy as np
import torch

from ..models.bert import BertEncoder, pack_for_encoder
from ..models.configs import decoder_config, encoder_config
from ..models.llama import LlamaDecoder, TPContext
from ..models.tokenizer import ChatFormat, decoder_tokenizer, encoder_tokenizer
from ..ops import h2d
from ..text.preprocess import extract_summary, preprocess_text
from . import prompts as P
from .generator import Generator


class Prompts(list):
    """A level of a summary plan: its prompts, and the tokens to generate for each (``max_new``)."""

    def __init__(self, prompts, max_new: int):
        super().__init__(prompts)
        self.max_new = max_new


class Engine:
    def __init__(self, embed_arch: str = "bge-base", llm_arch: str = "phi3-mini", device="cuda", seed: int = 0,
                 tp: TPContext | None = None, max_batch: int = 64, max_seq: int = 4096, temperature: float = 0.2,
                 max_new_tokens: int = 64, summary_max_new: int = 128, index_kind: str = "flat",
                 ivf_lists: int = 100, ivf_probes: int = 1, load_llm: bool = True, load_encoder: bool = True,
                 use_graphs: bool = True, embed_max_tokens: int = 65536, enc_dtype: str = "bf16",
                 share_prefix: bool = True, overlap_waves: bool = False, kv_cache_gb: float = 0.0):
        self.device = torch.device(device)
        self.lock = threading.RLock()      # the decoder / generator (one GPU thread drives it)
        self.enc_lock = threading.RLock()  # the encoder: the fast embed lane and the batcher share it
        self.enc_cfg = encoder_config(embed_arch)
        self.dec_cfg = decoder_config(llm_arch)
        self.enc_tok = encoder_tokenizer(self.enc_cfg.vocab)
        self.dec_tok = decoder_tokenizer(self.dec_cfg.vocab)
        self.chat = ChatFormat(self.dec_tok)
        self.temperature = temperature
        self.max_new_tokens = max_new_tokens
        self.summary_max_new = summary_max_new
        self.embed_max_tokens = embed_max_tokens
        # one short text (a question) through the encoder's captured length-bucket graphs,
        # captured here at startup rather than under the first request
        self.enc_graphs = use_graphs and self.device.type == "cuda"
        self.encoder = BertEncoder(self.enc_cfg, self.device, seed=seed, dtype=enc_dtype) if load_encoder else None
        if self.encoder is not None and self.enc_graphs:
            self.encoder.prepare_graphs()
        self.decoder = None
        self.gen = None
        if load_llm:
            self.decoder = LlamaDecoder(self.dec_cfg, self.device, seed=seed, tp=tp)
            if max_batch <= 0:
                max_batch = self.auto_batch(max_seq, overlap_waves, kv_gb=kv_cache_gb)
            # + 1 dummy slot (padded graph rows) + 2 prompt-head slots (ContinuousScheduler heads)
            # + 1 for the wave path's kept prompt head (Generator.head); overlap_waves: a second
            # wave's rows (answer_overlapped keeps two waves in flight)
            self.decoder.alloc_cache((2 if overlap_waves else 1) * max_batch + 4, max_seq)
            self.gen = Generator(self.decoder, max_batch=max_batch, max_seq=max_seq, temperature=temperature,
                                 seed=seed, eos=sorted(self.chat.eos_ids), use_graphs=use_graphs,
                                 share_prefix=share_prefix)
        from ..index import make_index
        self.index = make_index(index_kind, self.enc_cfg.hidden, self.device, lists=ivf_lists, probes=ivf_probes)
        self._prefix_cache: dict[str, list[int]] = {}
        self.stats = {"embed_texts": 0, "embed_tokens": 0, "embed_s": 0.0, "embed_truncated_texts": 0,
                      "embed_truncated_tokens": 0}

    AUTO_BATCH_MAX = 128            # decode rows: the deploy stack's measured best (profiles/r6/stack)
    AUTO_RESERVE_BYTES = 48 << 30  # HBM left beside the KV cache: index growth, activations, graphs

    def auto_batch(self, max_seq: int, overlap: bool = False, kv_gb: float = 0.0) -> int:
        """``max_batch=0``: the largest power-of-two decode batch (<= AUTO_BATCH_MAX) whose KV cache
        (batch + 4 slots x max_seq, this rank's kv heads) fits ``kv_gb`` GB, or the device's free
        HBM after the weights less AUTO_RESERVE_BYTES. Phi-3-mini on an MI355X: 128 (213 GB of
        KV); Llama-3-70B on one GPU: 16. CPU: 64."""
        from ..models.llama import KVCache
        if self.device.type != "cuda" and kv_gb <= 0:
            return 64
        per = KVCache.bytes_for(self.dec_cfg, 1, min(max_seq, self.dec_cfg.max_pos), self.decoder.tp.size)
        if kv_gb > 0:
            budget = int(kv_gb * 1e9)
        else:
            free, _ = torch.cuda.mem_get_info(self.device)
            budget = free - self.AUTO_RESERVE_BYTES
        b = self.AUTO_BATCH_MAX
        while b > 1 and ((2 if overlap else 1) * b + 4) * per > budget:
            b //= 2
        return b

    @property
    def dim(self) -> int:
        return self.enc_cfg.hidden

    # ------------------------------------------------------------------ embeddings
    def embed(self, texts: list[str], preprocess: bool = True, out_dtype=torch.bfloat16) -> torch.Tensor:
        """Unit-norm embeddings [n, d] on the engine device (1:1 with ``texts``)."""
        if self.encoder is None:
            raise RuntimeError("encoder not loaded")
        if preprocess:
            texts = [preprocess_text(t) for t in texts]
        n = len(texts)
        out = torch.empty((n, self.dim), dtype=out_dtype, device=self.device)
        if n == 0:
            return out
        t0 = time.perf_counter()
        trunc0 = (self.stats["embed_truncated_texts"], self.stats["embed_truncated_tokens"])
        seqs = pack_for_encoder(self.enc_tok, texts, self.enc_cfg.max_pos, self.stats)
        if self.stats["embed_truncated_texts"] != trunc0[0]:
            from ..utils import metrics
            metrics.ENGINE_EMBED_TRUNCATED.labels("texts").inc(self.stats["embed_truncated_texts"] - trunc0[0])
            metrics.ENGINE_EMBED_TRUNCATED.labels("tokens").inc(self.stats["embed_truncated_tokens"] - trunc0[1])
        if n == 1 and self.enc_graphs:
            with self.enc_lock:
                out[0] = self.encoder.encode_one(seqs[0])[0].to(out_dtype)
            self.stats["embed_tokens"] += len(seqs[0])
            self.stats["embed_texts"] += 1
            self.stats["embed_s"] += time.perf_counter() - t0
            return out
        if self.enc_graphs and n <= 64:  # a micro-batch of questions: one captured graph
            with self.enc_lock:
                v = self.encoder.encode_batch(seqs)
            if v is not None:
                out.copy_(v.to(out_dtype))
                self.stats["embed_tokens"] += sum(len(q) for q in seqs)
                self.stats["embed_texts"] += n
                self.stats["embed_s"] += time.perf_counter() - t0
                return out
        order = np.argsort([-len(s) for s in seqs], kind="stable")
        with self.enc_lock:
            i = 0
            while i < n:
                j, tot = i, 0
                while j < n and (j == i or tot + len(seqs[order[j]]) <= self.embed_max_tokens):
                    tot += len(seqs[order[j]])
                    j += 1
                idx = order[i:j]
                vec = self.encoder.encode_packed([seqs[k] for k in idx])
                out[h2d(idx, self.device)] = vec.to(out_dtype)
                self.stats["embed_tokens"] += tot
                i = j
        self.stats["embed_texts"] += n
        self.stats["embed_s"] += time.perf_counter() - t0
        return out

    def embed_one(self, text: str) -> torch.Tensor:
        """Embed(text): error on empty-after-preprocessing input (openai.go:44-47)."""
        t = preprocess_text(text)
        if not t:
            raise ValueError("text is empty after preprocessing")
        return self.embed([t], preprocess=False, out_dtype=torch.float32)[0]

    # ------------------------------------------------------------------ generation
    def _ids(self, s: str) -> list[int]:
        return self.dec_tok.encode(s, add_special_tokens=False).ids

    def _ids_many(self, texts: list[str]) -> list[list[int]]:
        """Batch tokenization (the tokenizer's thread pool): 64 2000-word documents take 250 ms
        one ``encode`` at a time on the GPU box's CPU share, ~10 % of an ingest batch
        (bench/tok_timing.py)."""
        if len(texts) <= 1:
            return [self._ids(t) for t in texts]
        return [e.ids for e in self.dec_tok.encode_batch(texts, add_special_tokens=False)]

    def _cached_ids(self, s: str) -> list[int]:
        v = self._prefix_cache.get(s)
        if v is None:
            v = self._ids(s)
            self._prefix_cache[s] = v
        return v

    def context_budget(self, max_new: int) -> int:
        return self.gen.cache.max_seq - max_new - 8

    def _answer_tail(self, question: str) -> str:
        return f"\nQuestion: {question}<|end|>\n<|assistant|>\n"

    def answer_prompt_ids(self, question: str, chunk_ids: list[list[int]], max_new: int,
                          tail: list[int] | None = None) -> list[int]:
        """Chat prompt for Answer with pre-tokenized chunks (tokenized once at ingest). Drops the
        lowest-ranked chunks first when the prompt would not fit the context.
        ``tail``: the question turn already tokenized (answer_many tokenizes a batch at once)."""
        head = self._cached_ids(f"<|system|>\n{P.ANSWER_SYSTEM}<|end|>\n<|user|>\nContext:\n")
        nl = self._cached_ids("\n")
        if tail is None:
            tail = self._ids(self._answer_tail(question))
        budget = self.context_budget(max_new) - len(head) - len(tail)
        ctx: list[int] = []
        for c in chunk_ids:
            if len(ctx) + len(c) + len(nl) > budget:
                break
            ctx.extend(c)
            ctx.extend(nl)
        return head + ctx + tail

    def answer_many(self, items, max_new: int | None = None):
        """items: (question, [chunk token-id lists ranked by score], context_quality) ->
        [(answer, confidence)] with confidence = quality * mean token probability."""
        max_new = max_new or self.max_new_tokens
        tails = self._ids_many([self._answer_tail(q) for q, _, _ in items])
        prompts = [self.answer_prompt_ids(q, ch, max_new, tail=t) for (q, ch, _), t in zip(items, tails)]
        with self.lock:
            res = self.gen.generate(prompts, max_new)
        texts = self.chat.decode_many([r.tokens for r in res])
        return [(txt, float(quality) * r.mean_prob) for (_, _, quality), r, txt in zip(items, res, texts)]

    def answer_overlapped(self, next_items, max_new: int | None = None, decode_frac: float = 0.5):
        """Waves of answers, the decode of one beside the prefill of the next (Generator.
        generate_overlapped; the engine must be built with overlap_waves=True). next_items(i) ->
        the items of wave i (answer_many's items) or None after the last; it runs while the previous
        wave decodes. decode_frac: the decode lane's share of the CUs (ops/streams.py lane_streams;
        0.5 measured best, profiles/r3/corun_expand.jsonl). Returns one answer_many result per wave."""
        from ..ops.streams import lane_streams
        max_new = max_new or self.max_new_tokens
        lanes = lane_streams(decode_frac, self.device)
        waves: list = []

        def next_prompts(i):
            items = next_items(i)
            if items is None:
                return None
            waves.append(items)
            tails = self._ids_many([self._answer_tail(q) for q, _, _ in items])
            return [self.answer_prompt_ids(q, ch, max_new, tail=t) for (q, ch, _), t in zip(items, tails)]
        with self.lock:
            res = self.gen.generate_overlapped(next_prompts, max_new, lanes)
        out = []
        for items, r in zip(waves, res):
            texts = self.chat.decode_many([x.tokens for x in r])
            out.append([(txt, float(q) * x.mean_prob) for (_, _, q), x, txt in zip(items, r, texts)])
        return out

    # ------------------------------------------------------------------ continuous batching
    @property
    def scheduler(self):
        """Lazily built ContinuousScheduler sharing this engine's generator and KV cache."""
        if getattr(self, "_sched", None) is None:
            from .generator import ContinuousScheduler
            self._sched = ContinuousScheduler(self.gen, B=self.gen.max_batch,
                                              max_new_cap=max(self.max_new_tokens, self.summary_max_new),
                                              max_admit_tokens=getattr(self, "admit_tokens", None))
        return self._sched

    def cb_tick(self, new_items, steps: int | None = None, stop=None):
        """Submit new work and run one scheduler tick. An item is ``(tag, (question, chunk_ids,
        quality))`` (an Answer) or ``(tag, {"ids": prompt_ids, "max_new": n})`` (a prebuilt prompt:
        summary windows). Returns ([(tag, text, confidence)], still_busy); a prompt item's
        confidence is its mean token probability."""
        sch = self.scheduler
        for tag, it in new_items:
            if isinstance(it, dict):
                sch.submit(it["ids"], int(it.get("max_new") or self.summary_max_new), (tag, 1.0))
            else:
                q, ch, quality = it
                sch.submit(self.answer_prompt_ids(q, ch, self.max_new_tokens), self.max_new_tokens, (tag, quality))
        with self.lock:
            done = sch.tick(steps, stop)
        out = [(tag, self.chat.decode(r.tokens), float(quality) * r.mean_prob) for (tag, quality), r in done]
        return out, sch.busy()

    def answer_text(self, question: str, context: str, quality: float, max_new: int | None = None):
        """Answer(ctx, question, contextText, contextQuality) with an untokenized context string."""
        max_new = max_new or self.max_new_tokens
        ids = self._ids(context)
        return self.answer_many([(question, [ids], quality)], max_new)[0] if ids else \
            self.answer_many([(question, [], quality)], max_new)[0]

    def _summary_frame(self, max_new: int):
        head = self._cached_ids(f"<|system|>\n{P.SUMMARIZE_SYSTEM}<|end|>\n<|user|>\n")
        tail = self._cached_ids("<|end|>\n<|assistant|>\n")
        return head, tail, self.context_budget(max_new) - len(head) - len(tail)

    def summary_windows(self, texts: list[str], max_new: int | None = None):
        """Map step of summarize: one prompt per text, or one per context-sized window of a text
        longer than the decoder context. Returns (prompts, owner) with owner[j] = (text index,
        is_partial). CPU only (tokenization), so the server runs it off the GPU thread."""
        head, tail, budget = self._summary_frame(max_new or self.summary_max_new)
        windows, owner = [], []
        for i, ids in enumerate(self._ids_many(list(texts))):
            if len(ids) <= budget:
                windows.append(head + ids + tail)
                owner.append((i, False))
            else:
                for s in range(0, len(ids), budget):
                    windows.append(head + ids[s:s + budget] + tail)
                    owner.append((i, True))
        return windows, owner

    def _reduce_groups(self, parts: list[str], budget: int) -> list[list[int]]:
        """One reduce level of one text: the summaries ``parts`` (window order), each tokenized on its
        own, packed in order into groups whose joined tokens (newline separated) fit ``budget``.
        Nothing is cut: a summary longer than half the budget is split into consecutive pieces of at
        most half the budget, so any two neighbours fit one group, every group but the last holds at
        least two pieces, and each level at least halves the pieces. Returns the groups' joined ids."""
        nl = self._cached_ids("\n")
        cap = (budget - len(nl)) // 2
        if cap < 1:
            raise ValueError(f"summary reduce: context budget {budget} too small to join two summaries")
        pieces: list[list[int]] = []
        for ids in self._ids_many(list(parts)):
            if not ids:
                continue
            pieces.extend(ids[s:s + cap] for s in range(0, len(ids), cap))
        groups: list[list[int]] = []
        cur: list[int] = []
        for pc in pieces:
            if cur and len(cur) + len(nl) + len(pc) > budget:
                groups.append(cur)
                cur = []
            cur = cur + nl + pc if cur else list(pc)
        if cur or not groups:
            groups.append(cur)
        return groups

    def summary_plan(self, texts: list[str], max_new: int | None = None):
        """Map-reduce summarization as a plan: a generator that yields lists of
        prompts (token ids) and is sent back their generated texts in the same order; its return
        value is the final raw summary of each text. The reference sends the whole document to a
        128k-context model in one request (cmd/analysis/main.go:70-71, internal/llm/openai.go:40-62);
        here a text longer than the decoder context is summarized per context-sized window (map),
        then its window summaries are reduced LEVEL BY LEVEL: each level packs the previous level's
        summaries, in order, into as few context-sized prompts as hold them all
        (``_reduce_groups``), until one prompt holds them — every window reaches the final summary,
        nothing is truncated. ``summarize_many`` drives it with the wave generator, the engine
        server with the continuous scheduler."""
        max_new = max_new or self.summary_max_new
        head, tail, _ = self._summary_frame(max_new)
        # reduce levels converge only if a generated summary (re-tokenized) fits half a reduce
        # prompt's budget: with budget = max_seq - new - 8 - head - tail, that needs
        # new <= (budget - 1) / 2, i.e. 3 * new <= max_seq - 9 - head - tail. A max_new above that
        # (a short context, a long summary setting) generates the reduce levels with the largest
        # budget that converges (10 % slack for re-tokenization) instead of never converging
        fit = int(0.9 * (self.gen.cache.max_seq - 9 - len(head) - len(tail)) // 3)
        if fit < 1:
            raise ValueError(f"summary reduce: decoder context {self.gen.cache.max_seq} too small")
        reduce_new = min(max_new, fit)
        budget = self.context_budget(reduce_new) - len(head) - len(tail)
        windows, owner = self.summary_windows(texts, max_new)
        outs = yield Prompts(windows, max_new)
        final: dict[int, str] = {}
        pending: dict[int, list[str]] = {}
        for (i, is_part), txt in zip(owner, outs):
            if is_part:
                pending.setdefault(i, []).append(txt)
            else:
                final[i] = txt
        levels = 0
        while pending:
            levels += 1
            if levels > 64:
                raise RuntimeError("summary reduce did not converge")
            prompts, pown = [], []  # pown[j] = (text index, final level?)
            for i, parts in pending.items():
                groups = self._reduce_groups(parts, budget)
                for g in groups:
                    prompts.append(head + g + tail)
                    pown.append((i, len(groups) == 1))
            outs = yield Prompts(prompts, reduce_new)
            nxt: dict[int, list[str]] = {}
            for (i, last), txt in zip(pown, outs):
                if last:
                    final[i] = txt
                else:
                    nxt.setdefault(i, []).append(txt)
            pending = nxt
        self.stats["summary_reduce_levels_max"] = max(self.stats.get("summary_reduce_levels_max", 0), levels)
        return [final[i] for i in range(len(texts))]

    @staticmethod
    def summary_step(plan, outs=None):
        """Advance a ``summary_plan``: ("prompts", [ids]) to generate next, or ("done", [text]).
        (A plain call, so it can run on an executor thread: StopIteration must not cross a future.)"""
        try:
            return "prompts", (next(plan) if outs is None else plan.send(outs))
        except StopIteration as e:
            return "done", e.value

    def summarize_many(self, texts: list[str], max_new: int | None = None) -> list[tuple[str, list[str]]]:
        """Summarize each text (map-reduce over the decoder context for long ones: ``summary_plan``)."""
        max_new = max_new or self.summary_max_new
        plan = self.summary_plan(texts, max_new)
        kind, val = self.summary_step(plan)
        while kind == "prompts":
            with self.lock:
                res = self.gen.generate(val, getattr(val, "max_new", max_new))
            kind, val = self.summary_step(plan, self.chat.decode_many([r.tokens for r in res]))
        return [extract_summary(t) for t in val]

    def release_decoder(self) -> dict:
        """Drop the decoder's KV cache, decode states and captured graphs (the weights stay: the
        N > 1 bench blocks shard them). Returns the generator's final stats. After this the engine
        can still embed and search but no longer generate. bench.py calls it before building the
        tensor-parallel decoders of its N > 1 blocks, whose caches would not fit beside this one
        (parallel/hbm_plan.py: 213 GB for 132 x 4096 Phi-3 slots)."""
        if self.gen is None:
            return {}
        with self.lock:
            stats = dict(self.gen.stats)
            if getattr(self, "_sched", None) is not None:
                self._sched = None
            self.gen.close()
            self.gen = None
            if self.decoder is not None:
                self.decoder.cache = None
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
            torch.cuda.empty_cache()  # the xGMI buffers are hipMalloc'd outside the caching allocator
        return stats

    # ------------------------------------------------------------------ introspection
    def describe(self) -> dict:
        d = {"encoder": self.enc_cfg.name, "decoder": self.dec_cfg.name, "device": str(self.device),
             "dim": self.dim, "index": self.index.kind, "index_rows": len(self.index)}
        if self.gen is not None:
            d["gen"] = dict(self.gen.stats)
            if getattr(self, "_sched", None) is not None:
                d["sched"] = dict(self._sched.stats)
        d["embed"] = dict(self.stats)
        return d
