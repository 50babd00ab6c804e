"""Llama-3 / Phi-3 decoder on the gfx950 kernels, with Megatron-style tensor parallelism over RCCL.

Replaces gpt-4o-mini for ``Summarize`` and ``Answer`` (internal/llm/openai.go:40-105; SURVEY.md §2.4
N6-N8). Per layer (hidden state x is the residual stream, updated in place):

    h   = RMSNorm(x)                                   rmsnorm kernel
    qkv = h @ Wqkv^T                                   MFMA GEMM   (column-parallel: local heads)
    RoPE(q, k) + write k, v to the KV cache            prefill: the GEMM's epilogue; decode: the
                                                       attention kernel (MHA) / rope_cache (GQA)
    a   = attention(q, K, V)                           varlen flash prefill / split-KV decode
    x   = x + a @ Wo^T                                 GEMM + fused residual epilogue (row-parallel
                                                       -> RCCL all-reduce over xGMI when TP > 1)
    h   = RMSNorm(x)
    g   = silu(h Wg^T) * (h Wu^T)                      ONE GEMM with the fused SwiGLU epilogue
    x   = x + g @ Wdown^T                              GEMM + residual (row-parallel + all-reduce)

TP layout (rank r of t): local q/k/v heads, F/t FFN features, vocab-parallel lm_head. Generation
never gathers the [B, V/t] logits: each rank reduces its slice to 8 floats per row (best Gumbel
score + its global index, local max, local sum-exp, the best's logit) and one tiny gather of those
picks the token and its full-vocabulary logprob (distributed sampling, SURVEY §2.4 C4;
``LlamaDecoder.sample``). With TP the residual is added by rank 0's epilogue only, so a single
in-place all-reduce yields x + sum of partials.
"""
from __future__ import annotations

import numpy as np
import torch

from ..ops import get_ops
from ..ops.reference import interleave_gate_up, rope_table
from .configs import DecoderConfig

EPI_NONE, EPI_SWIGLU, EPI_RESID, EPI_ROPE = 0, 3, 4, 6
# Decode step of MHA models: RoPE + KV-cache write folded into the attention kernel (False: separate
# rope_cache launch; the GPU tests compare both).
_FUSED_ROPE_DECODE = True


class TPContext:
    """Tensor-parallel process group (identity when size == 1)."""

    def __init__(self, rank: int = 0, size: int = 1, group=None, xgmi: bool = True):
        self.rank, self.size, self.group = rank, size, group
        self.use_xgmi = xgmi  # False: every all-reduce / gather through torch.distributed (RCCL)
        self.xgmi = None  # XgmiAllReduce once setup_device() ran on a GPU
        self.xgmi_norm = None  # a second communicator for the fused all-reduce + RMSNorm (one row width)

    def setup_device(self, device: torch.device) -> None:
        """Collective (every TP rank): map the peers' all-reduce buffers over xGMI (GPU only).
        Decode-sized row-parallel outputs then take the one-/two-shot IPC kernel; anything else
        (and every CPU run) uses torch.distributed (RCCL / gloo)."""
        if self.size > 1 and device.type == "cuda" and self.xgmi is None and self.use_xgmi:
            from ..parallel.xgmi_allreduce import XgmiAllReduce
            self.xgmi = XgmiAllReduce.create(self.group, device)
            if self.xgmi is not None:
                # decode-sized rows only (one-shot): 512 KB = 32 rows of Llama-3-70B's 8192
                self.xgmi_norm = XgmiAllReduce.create(self.group, device, max_bytes=512 << 10)

    def close(self) -> None:
        """Collective (every TP rank): release the xGMI communicators once no rank uses them any more
        (a process that builds several TP models, e.g. bench.py's N > 1 blocks, would otherwise keep
        every model's IPC-exported buffers mapped on every peer)."""
        comms = [c for c in (self.xgmi, self.xgmi_norm) if c is not None]
        if not comms:
            return
        import torch.distributed as dist
        dist.barrier(group=self.group)
        for c in comms:
            c.close()
        self.xgmi = self.xgmi_norm = None

    def all_reduce_(self, t: torch.Tensor) -> torch.Tensor:
        if self.size > 1:
            if self.xgmi is not None and self.xgmi.takes(t):
                return self.xgmi.all_reduce_(t)
            import torch.distributed as dist
            if t.is_cuda and dist.get_backend(self.group) == "gloo":  # 1-GPU multi-rank rehearsal
                h = t.cpu()
                dist.all_reduce(h, group=self.group)
                t.copy_(h)
            else:
                dist.all_reduce(t, group=self.group)
        return t

    def all_reduce_norm_(self, x: torch.Tensor, gamma, eps: float, h_out: torch.Tensor, ops) -> torch.Tensor:
        """x <- sum over the group (in place), h_out <- RMSNorm(x) * gamma. One fused launch over
        the xGMI peer buffers when it takes the rows (C3 with the residual stream's next norm in its
        epilogue); otherwise the all-reduce and the rmsnorm kernel (CPU / gloo: the same math)."""
        if self.size > 1 and self.xgmi_norm is not None and self.xgmi_norm.takes_norm(x):
            return self.xgmi_norm.all_reduce_rmsnorm_(x, gamma, eps, h_out)
        self.all_reduce_(x)
        return ops.rmsnorm(x, gamma, eps, out=h_out)

    def all_gather_cols(self, t: torch.Tensor) -> torch.Tensor:
        """[B, n] on every rank -> [B, n * size] (rank-major columns)."""
        if self.size == 1:
            return t
        if self.xgmi is not None:
            # over the peer-mapped xGMI buffers (graph-capturable, unlike a host-staged gather):
            # every rank contributes its columns into a zero [B, n * size] row block and the
            # one-shot all-reduce sums them; x + 0 is exact, so this IS the all-gather
            B, n = t.shape
            full = torch.zeros((B, n * self.size), dtype=t.dtype, device=t.device)
            full[:, self.rank * n:(self.rank + 1) * n] = t
            if self.xgmi.takes(full):
                return self.xgmi.all_reduce_(full)
        from ..parallel.dist import all_gather_rows
        out = all_gather_rows(t.contiguous(), self.group)
        return out.view(self.size, t.shape[0], -1).permute(1, 0, 2).reshape(t.shape[0], -1)


def tp_sample(ops, tp: TPContext, logits, temperature: float, seed: int, step: int = 0, **kw):
    """Sampling over a vocab-parallel LM head (see LlamaDecoder.sample): partial stats of this rank's
    slice [B, V/t] (global indices from rank * V/t), one all-gather of [B, 8] fp32, finalize."""
    if tp.size == 1:
        return ops.sample(logits, temperature, seed, step, **kw)
    ctr = kw.pop("ctr", None)
    stats = ops.sample_partial(logits, temperature, seed, v0=tp.rank * logits.shape[1], step=step, ctr=ctr)
    gathered = tp.all_gather_cols(stats).contiguous()
    return ops.sample_finalize(gathered, tp.size, **kw)


def to_interleaved_rope(wqkv: torch.Tensor, H: int, Hkv: int, D: int) -> torch.Tensor:
    """Convert an HF (rotate_half: pairs (i, i + D/2)) QKV weight to this engine's interleaved RoPE
    layout (pairs (2i, 2i + 1)) by permuting the rows of every q and k head; v rows are unchanged.
    q.k is invariant under the same permutation of both, so attention outputs are identical."""
    perm = torch.stack([torch.arange(D // 2), torch.arange(D // 2) + D // 2], dim=1).flatten()
    qk = wqkv[:(H + Hkv) * D].view(H + Hkv, D, -1)[:, perm.to(wqkv.device)].reshape((H + Hkv) * D, -1)
    return torch.cat([qk, wqkv[(H + Hkv) * D:]]).contiguous()


def _randn(shape, gen, device, std=0.02):
    t = torch.empty(shape, dtype=torch.float32, device=device)
    t.normal_(0.0, std, generator=gen)
    return t.to(torch.bfloat16)


def shard_weights(cfg: DecoderConfig, full: dict, rank: int, size: int) -> dict:
    """Slice a full (unsharded) weight dict for TP rank ``rank`` of ``size``."""
    if size == 1:
        return full
    H, Hkv, D, F, V = cfg.heads, cfg.kv_heads, cfg.head_dim, cfg.ffn, cfg.vocab
    assert H % size == 0 and Hkv % size == 0 and F % (16 * size) == 0 and V % size == 0
    hl, kl, fl, vl = H // size, Hkv // size, F // size, V // size
    out = {"embed": full["embed"], "norm": full["norm"],
           "lm_head": full["lm_head"][rank * vl:(rank + 1) * vl].contiguous(), "layers": []}
    for L in full["layers"]:
        q = L["wqkv"][:H * D].view(H, D, -1)[rank * hl:(rank + 1) * hl].reshape(hl * D, -1)
        k = L["wqkv"][H * D:(H + Hkv) * D].view(Hkv, D, -1)[rank * kl:(rank + 1) * kl].reshape(kl * D, -1)
        v = L["wqkv"][(H + Hkv) * D:].view(Hkv, D, -1)[rank * kl:(rank + 1) * kl].reshape(kl * D, -1)
        out["layers"].append({
            "wqkv": torch.cat([q, k, v]).contiguous(),
            "wo": L["wo"][:, rank * hl * D:(rank + 1) * hl * D].contiguous(),
            "w_gu": L["w_gu"][2 * rank * fl:2 * (rank + 1) * fl].contiguous(),
            "w_down": L["w_down"][:, rank * fl:(rank + 1) * fl].contiguous(),
            "ln_attn": L["ln_attn"], "ln_mlp": L["ln_mlp"],
        })
    return out


def random_weights(cfg: DecoderConfig, device, seed: int = 0, tp_rank: int = 0, tp_size: int = 1,
                   full_then_shard: bool = False) -> dict:
    """Seeded random init. Large models generate only the local TP shard (seeded per shard);
    ``full_then_shard`` builds the full model first (tests: TP result == unsharded result)."""
    dev = torch.device(device)
    if full_then_shard and tp_size > 1:
        return shard_weights(cfg, random_weights(cfg, device, seed), tp_rank, tp_size)
    gen = torch.Generator(device=dev)
    gen.manual_seed(seed * 1_000_003 + 101)  # shared part (embedding, norms) identical on all ranks
    h, D, F, V = cfg.hidden, cfg.head_dim, cfg.ffn, cfg.vocab
    hl, kl, fl, vl = cfg.heads // tp_size, cfg.kv_heads // tp_size, F // tp_size, V // tp_size
    w = {"embed": _randn((V, h), gen, dev), "norm": torch.ones(h, dtype=torch.bfloat16, device=dev), "layers": []}
    gen.manual_seed(seed * 1_000_003 + 7 * tp_rank + 1)
    std_o = 0.02 / (2 * cfg.layers) ** 0.5
    for _ in range(cfg.layers):
        gate = _randn((fl, h), gen, dev)
        up = _randn((fl, h), gen, dev)
        w["layers"].append({
            "wqkv": _randn(((hl + 2 * kl) * D, h), gen, dev),
            "wo": _randn((h, hl * D), gen, dev, std_o),
            "w_gu": interleave_gate_up(gate, up),
            "w_down": _randn((h, fl), gen, dev, std_o),
            "ln_attn": torch.ones(h, dtype=torch.bfloat16, device=dev),
            "ln_mlp": torch.ones(h, dtype=torch.bfloat16, device=dev),
        })
        del gate, up
    w["lm_head"] = _randn((vl, h), gen, dev)
    return w


class KVCache:
    """Contiguous per-slot KV cache: k/v [layers][slots, Hkv_local, max_seq, D] (one allocation)."""

    def __init__(self, cfg: DecoderConfig, slots: int, max_seq: int, tp_size: int, device):
        self.slots, self.max_seq = slots, max_seq
        self.hkv = cfg.kv_heads // tp_size
        self.buf = torch.zeros((cfg.layers, 2, slots, self.hkv, max_seq, cfg.head_dim), dtype=torch.bfloat16,
                               device=device)
        self.free = list(range(slots - 1, -1, -1))

    def k(self, layer):
        return self.buf[layer, 0]

    def v(self, layer):
        return self.buf[layer, 1]

    def acquire(self, n: int) -> list[int]:
        if n > len(self.free):
            raise RuntimeError(f"KV cache exhausted: want {n} slots, {len(self.free)} free")
        return [self.free.pop() for _ in range(n)]

    def release(self, ids):
        self.free.extend(ids)

    @staticmethod
    def bytes_for(cfg: DecoderConfig, slots: int, max_seq: int, tp_size: int = 1) -> int:
        return cfg.layers * 2 * slots * (cfg.kv_heads // tp_size) * max_seq * cfg.head_dim * 2


class LlamaDecoder:
    unit_gains = False  # set by _fold_norm_gains
    layer_hook = None   # prefill: called with the layer index before each layer (stream steering)

    def __init__(self, cfg: DecoderConfig, device="cuda", seed: int = 0, tp: TPContext | None = None,
                 weights: dict | None = None):
        self.cfg = cfg
        self.device = torch.device(device)
        self.ops = get_ops(self.device)
        self.tp = tp or TPContext()
        self.tp.setup_device(self.device)
        t = self.tp.size
        if cfg.heads % t or cfg.kv_heads % t:
            raise ValueError(f"TP={t} must divide heads={cfg.heads} and kv_heads={cfg.kv_heads}")
        self.hl, self.kl = cfg.heads // t, cfg.kv_heads // t
        self.w = weights if weights is not None else random_weights(cfg, self.device, seed, self.tp.rank, t)
        self._fold_norm_gains()
        self.cos_sin = rope_table(cfg.max_pos, cfg.head_dim, cfg.rope_theta, self.device)
        self.cache: KVCache | None = None

    def _fold_norm_gains(self):
        """Fold every RMSNorm gain into the weights that consume the normalised rows (W -> W diag(g),
        then g = 1): the same model, and the batch-1 GEMVs fuse the norm without streaming a gain
        vector next to the weights (rms=(None, eps)). Random-init gains are already 1; converted
        checkpoints are folded here, once."""
        pairs = [(L, "ln_attn", "wqkv") for L in self.w["layers"]] + [(L, "ln_mlp", "w_gu") for L in self.w["layers"]]
        pairs.append((self.w, "norm", "lm_head"))
        for d, gk, wk in pairs:
            g = d[gk]
            if not bool(torch.all(g == 1)):
                d[wk] = (d[wk].float() * g.float()[None, :]).to(d[wk].dtype).contiguous()
                d[gk] = torch.ones_like(g)
        self.unit_gains = True

    def _gain(self, g):
        """The gain a fused batch-1 GEMV norm streams: none once the gains are folded."""
        return None if self.unit_gains else g

    def alloc_cache(self, slots: int, max_seq: int) -> KVCache:
        max_seq = min(max_seq, self.cfg.max_pos)
        self.cache = KVCache(self.cfg, slots, max_seq, self.tp.size, self.device)
        return self.cache

    # ------------------------------------------------------------- shared layer body
    def _attn_out_and_mlp(self, L, a, x):
        o, tp = self.ops, self.tp
        if tp.size == 1 or tp.rank == 0:
            o.gemm(a, L["wo"], epi=EPI_RESID, resid=x, out=x)
        else:
            o.gemm(a, L["wo"], out=x)
        tp.all_reduce_(x)
        return self._mlp(L, x)

    def _mlp(self, L, x):
        o, tp = self.ops, self.tp
        if o.gemv_fusable(x.shape[0], L["w_gu"].shape[0], x.shape[1], EPI_SWIGLU):  # batch 1: norm fused
            g = o.gemm(x, L["w_gu"], epi=EPI_SWIGLU, rms=(self._gain(L["ln_mlp"]), self.cfg.eps))
        else:
            h = o.rmsnorm(x, L["ln_mlp"], self.cfg.eps)
            g = o.gemm(h, L["w_gu"], epi=EPI_SWIGLU)
        if tp.size == 1 or tp.rank == 0:
            o.gemm(g, L["w_down"], epi=EPI_RESID, resid=x, out=x)
        else:
            o.gemm(g, L["w_down"], out=x)
        tp.all_reduce_(x)
        return x

    def _logits(self, hlast, gather: bool = True, out=None):
        """Logits of the rows of ``hlast``: the full [B, V] (gather=True; an all-gather of the vocab
        slices under TP) or this rank's slice [B, V/t] (gather=False: what ``sample`` consumes;
        ``out`` receives it)."""
        o = self.ops
        if o.gemv_fusable(hlast.shape[0], self.w["lm_head"].shape[0], hlast.shape[1]):
            logits = o.gemm(hlast.contiguous(), self.w["lm_head"], rms=(self._gain(self.w["norm"]), self.cfg.eps),
                            out=None if gather else out)
        else:
            h = o.rmsnorm(hlast, self.w["norm"], self.cfg.eps)
            logits = o.gemm(h, self.w["lm_head"], out=None if gather else out)
        return self.tp.all_gather_cols(logits) if gather else logits

    def sample(self, logits, temperature: float, seed: int, step: int = 0, **kw):
        """Sample one token per row from this rank's logits (the full row at TP=1, its vocab slice
        under TP) with the fused sampler's bookkeeping (``ops.sample`` keywords). Under TP: the
        slice's 8-float summary per row -> ONE all-gather of [B, 8] fp32 per rank (graph-capturable
        over the xGMI peer buffers) -> the finalize kernel; every rank ends with the same token,
        logprob and bookkeeping, identical to sampling the gathered row."""
        return tp_sample(self.ops, self.tp, logits, temperature, seed, step, **kw)

    # ------------------------------------------------------------- prefill
    def prefill(self, ids: torch.Tensor, pos: torch.Tensor, slot_tok: torch.Tensor, cu: torch.Tensor,
                max_seqlen: int, last_idx: torch.Tensor, prefix: tuple[int, int] | None = None,
                local_logits: bool = False) -> torch.Tensor:
        """Packed causal prefill; writes the KV cache; returns logits [B, V] of each sequence's last token
        (local_logits: this rank's vocab slice [B, V/t], the input of ``sample``).
        prefix = (slot, P): every sequence continues a shared P-token head already in ``slot``'s cache
        (``pos`` then starts at P); attention reads those keys from the cache."""
        c, o, cache = self.cfg, self.ops, self.cache
        D, hl, kl = c.head_dim, self.hl, self.kl
        x = o.embed(ids, self.w["embed"])
        hook = self.layer_hook
        kv_from_cache = bool(getattr(o, "flash_kv_cache_ok", lambda *_: False)(D, True))
        for li, L in enumerate(self.w["layers"]):
            if hook is not None:  # e.g. move the rest of a prefill to another (CU-masked) stream
                hook(li)
            h = o.rmsnorm(x, L["ln_attn"], c.eps)
            # QKV projection + RoPE + KV-cache write in one kernel (gemm8p EPI_ROPE epilogue); where the
            # attention reads its keys from the cache (Phi-3's D = 96), k / v go to the cache only
            qkv = o.gemm_rope(h, L["wqkv"], pos, self.cos_sin, hl, kl, D, slot_tok, cache.k(li), cache.v(li),
                              kv_out=not kv_from_cache)
            pre = None if prefix is None else (cache.k(li)[prefix[0]], cache.v(li)[prefix[0]], prefix[1])
            if kv_from_cache:
                a = o.flash_attn_varlen(qkv[:, :hl * D], None, None, cu, max_seqlen, hl, kl, D, causal=True,
                                        prefix=pre, kv_cache=(cache.k(li), cache.v(li), slot_tok, pos))
            else:
                a = o.flash_attn_varlen(qkv[:, :hl * D], qkv[:, hl * D:(hl + kl) * D], qkv[:, (hl + kl) * D:], cu,
                                        max_seqlen, hl, kl, D, causal=True, prefix=pre)
            del qkv, h
            x = self._attn_out_and_mlp(L, a, x)
        return self._logits(x.index_select(0, last_idx), gather=not local_logits)

    # ------------------------------------------------------------- decode (graph-capturable)
    def decode_step(self, st: "DecodeState") -> torch.Tensor:
        c, o, cache = self.cfg, self.ops, self.cache
        D, hl, kl = c.head_dim, self.hl, self.kl
        x = o.embed(st.tokens, self.w["embed"], out=st.x)
        if self._dk_decode(x.shape[0]):
            return self._decode_step_dk(st, x)
        if self._norm_fusable(x.shape[0]):
            return self._decode_step_fused_norms(st, x)
        if self.tp.size > 1 and x.shape[0] > 1:
            return self._decode_step_tp_fused_norms(st, x)
        fuse = o.gemv_fusable(x.shape[0], self.w["layers"][0]["wqkv"].shape[0], x.shape[1])
        for li, L in enumerate(self.w["layers"]):
            if fuse:  # batch 1: RMSNorm folded into the QKV GEMV (no separate norm launch)
                qkv = o.gemm(x, L["wqkv"], out=st.qkv, rms=(self._gain(L["ln_attn"]), c.eps))
            else:
                h = o.rmsnorm(x, L["ln_attn"], c.eps, out=st.h)
                qkv = o.gemm(h, L["wqkv"], out=st.qkv)
            a = self._decode_attn(qkv, li, st)
            self._attn_out_and_mlp(L, a, x)
        logits = self._logits(x, gather=False, out=st.logits)  # straight into the state (no copy launch)
        if logits.data_ptr() != st.logits.data_ptr():
            st.logits.copy_(logits)
        self.sample(st.logits, st.temperature, st.seed, 0, out_tok=st.tokens, out_lp=st.lp, conf=st.conf,
                    active=st.active, ctr=st.pos, pos=st.pos, lens=st.lens, hist=st.hist, start=st.start, eos=st.eos)
        return st.tokens

    def _decode_attn(self, qkv, li: int, st: "DecodeState"):
        """RoPE + new-token cache write + decode attention. MHA (Phi-3): one launch — the attention
        kernel rotates q / the new k itself and writes the new k / v to the cache; GQA: rope_cache,
        then the MFMA decode kernel."""
        c, o, cache = self.cfg, self.ops, self.cache
        D, hl, kl = c.head_dim, self.hl, self.kl
        if hl == kl and _FUSED_ROPE_DECODE:
            return o.decode_attn(qkv, cache.k(li), cache.v(li), st.lens, st.slot, hl, kl, D, max_len=cache.max_seq,
                                 pre=st.pre, rope=(self.cos_sin, st.pos), out=st.attn)
        o.rope_cache(qkv, st.pos, self.cos_sin, hl, kl, D, slot=st.slot, k_cache=cache.k(li), v_cache=cache.v(li))
        return o.decode_attn(qkv, cache.k(li), cache.v(li), st.lens, st.slot, hl, kl, D, max_len=cache.max_seq,
                             pre=st.pre, out=st.attn)

    def _norm_fusable(self, B: int) -> bool:
        """Batched decode (1 < B <= 128, no TP; B <= 64 normally takes gemm_dk first): every RMSNorm
        rides on the split-K reduction of the projection before it (gemm_resid_norm), so a layer is
        2 GEMM+reduce pairs, 2 plain GEMMs, RoPE/cache and attention — no standalone norm launches."""
        return self.tp.size == 1 and 1 < B <= 128 and self.cfg.hidden <= 8192 and self.cfg.hidden % 8 == 0

    def _dk_decode(self, B: int) -> bool:
        """Batched decode (2 <= B <= 64, no TP) on gemm_dk: every projection one launch without
        split-K partials, the RMSNorms deferred into the consuming GEMM (needs folded gains)."""
        o, c = self.ops, self.cfg
        f = getattr(o, "dk_fusable", None)
        if f is None or self.tp.size != 1 or not self.unit_gains or not 2 <= B <= 64:
            return False
        L = self.w["layers"][0]
        shapes = [(L["wqkv"], EPI_NONE), (L["wo"], EPI_RESID), (L["w_gu"], EPI_SWIGLU), (L["w_down"], EPI_RESID),
                  (self.w["lm_head"], EPI_NONE)]
        return all(f(B, w.shape[0], w.shape[1], e) for w, e in shapes) and o.dk_parts(c.hidden, B) <= 512

    def _decode_step_dk(self, st: "DecodeState", x: torch.Tensor) -> torch.Tensor:
        """A layer = QKV, attention, O (+ residual, row sums of squares), gate/up + SwiGLU (norm
        deferred from those sums), down (+ residual, sums): 5 launches, no reduce launches, no
        standalone norms after layer 0's input norm."""
        c, o = self.cfg, self.ops
        layers = self.w["layers"]
        sa, sb = st.ssq
        parts = o.dk_parts(c.hidden, x.shape[0])
        a_in, norm = o.rmsnorm(x, layers[0]["ln_attn"], c.eps, out=st.h), None
        for li, L in enumerate(layers):
            qkv = o.gemm_dk(a_in, L["wqkv"], out=st.qkv, norm_in=norm)
            a = self._decode_attn(qkv, li, st)
            o.gemm_dk(a, L["wo"], epi=EPI_RESID, resid=x, out=x, ssq_out=sa)               # x += o
            g = o.gemm_dk(x, L["w_gu"], epi=EPI_SWIGLU, norm_in=(sa, parts, c.eps))        # norm(x) -> gate/up
            o.gemm_dk(g, L["w_down"], epi=EPI_RESID, resid=x, out=x, ssq_out=sb)           # x += mlp
            a_in, norm = x, (sb, parts, c.eps)
        o.gemm_dk(x, self.w["lm_head"], out=st.logits, norm_in=norm)                      # final norm deferred
        o.sample(st.logits, st.temperature, st.seed, 0, out_tok=st.tokens, out_lp=st.lp, conf=st.conf,
                 active=st.active, ctr=st.pos, pos=st.pos, lens=st.lens, hist=st.hist, start=st.start, eos=st.eos)
        return st.tokens

    def _decode_step_fused_norms(self, st: "DecodeState", x: torch.Tensor) -> torch.Tensor:
        c, o, cache = self.cfg, self.ops, self.cache
        D, hl, kl = c.head_dim, self.hl, self.kl
        layers = self.w["layers"]
        h = o.rmsnorm(x, layers[0]["ln_attn"], c.eps, out=st.h)
        for li, L in enumerate(layers):
            qkv = o.gemm(h, L["wqkv"], out=st.qkv)
            a = self._decode_attn(qkv, li, st)
            h = o.gemm_resid_norm(a, L["wo"], x, L["ln_mlp"], c.eps, out=x, h_out=st.h)      # x += o; h = norm(x)
            g = o.gemm(h, L["w_gu"], epi=EPI_SWIGLU)
            nxt = layers[li + 1]["ln_attn"] if li + 1 < len(layers) else self.w["norm"]
            h = o.gemm_resid_norm(g, L["w_down"], x, nxt, c.eps, out=x, h_out=st.h)       # x += mlp; h = norm(x)
        st.logits.copy_(o.gemm(h, self.w["lm_head"]))  # h already carries the final norm
        o.sample(st.logits, st.temperature, st.seed, 0, out_tok=st.tokens, out_lp=st.lp, conf=st.conf,
                 active=st.active, ctr=st.pos, pos=st.pos, lens=st.lens, hist=st.hist, start=st.start, eos=st.eos)
        return st.tokens

    def _decode_step_tp_fused_norms(self, st: "DecodeState", x: torch.Tensor) -> torch.Tensor:
        """Tensor-parallel decode (B > 1) with the TP=1 fused-norm structure: every RMSNorm rides in
        the epilogue of the all-reduce before it (the o-proj's sum + ln_mlp, the down-proj's sum +
        the next layer's ln_attn / the final norm), so a layer is QKV GEMM, attention, o GEMM, fused
        AR+norm, gate/up GEMM, down GEMM, fused AR+norm — no standalone norm launches."""
        c, o, tp = self.cfg, self.ops, self.tp
        layers = self.w["layers"]
        h = o.rmsnorm(x, layers[0]["ln_attn"], c.eps, out=st.h)
        for li, L in enumerate(layers):
            qkv = o.gemm(h, L["wqkv"], out=st.qkv)
            a = self._decode_attn(qkv, li, st)
            if tp.rank == 0:
                o.gemm(a, L["wo"], epi=EPI_RESID, resid=x, out=x)
            else:
                o.gemm(a, L["wo"], out=x)
            h = tp.all_reduce_norm_(x, L["ln_mlp"], c.eps, st.h, o)
            g = o.gemm(h, L["w_gu"], epi=EPI_SWIGLU)
            if tp.rank == 0:
                o.gemm(g, L["w_down"], epi=EPI_RESID, resid=x, out=x)
            else:
                o.gemm(g, L["w_down"], out=x)
            nxt = layers[li + 1]["ln_attn"] if li + 1 < len(layers) else self.w["norm"]
            h = tp.all_reduce_norm_(x, nxt, c.eps, st.h, o)
        st.logits.copy_(o.gemm(h, self.w["lm_head"]))  # h already carries the final norm; local vocab slice
        self.sample(st.logits, st.temperature, st.seed, 0, out_tok=st.tokens, out_lp=st.lp, conf=st.conf,
                    active=st.active, ctr=st.pos, pos=st.pos, lens=st.lens, hist=st.hist, start=st.start, eos=st.eos)
        return st.tokens

    def prefill_flops(self, lens) -> float:
        c = self.cfg
        h, D = c.hidden, c.head_dim
        lin = 2 * (h * (c.heads + 2 * c.kv_heads) * D + c.heads * D * h + 3 * h * c.ffn)
        tot = 0.0
        for L in lens:
            tot += c.layers * (L * lin + 2 * c.heads * D * L * L) + 2 * h * c.vocab
        return tot


class DecodeState:
    """Static device buffers for a batch bucket of B sequences (HIP-graph friendly)."""

    def __init__(self, model: LlamaDecoder, B: int, max_new: int, temperature: float, seed: int, eos=()):
        c, dev = model.cfg, model.device
        i32 = dict(dtype=torch.int32, device=dev)
        self.B = B
        self.tokens = torch.zeros(B, **i32)
        self.pos = torch.zeros(B, **i32)
        self.lens = torch.ones(B, **i32)
        self.slot = torch.zeros(B, **i32)
        self.active = torch.zeros(B, **i32)
        self.start = torch.zeros(B, **i32)
        self.pre = torch.zeros(B, 2, **i32)  # (P, slot): shared prompt head of row b (decode_attn pre)
        self.hist = torch.full((B, max(1, max_new)), -1, **i32)
        self.conf = torch.zeros(B, 2, dtype=torch.float32, device=dev)
        self.lp = torch.zeros(B, dtype=torch.float32, device=dev)
        h = c.hidden
        self.x = torch.zeros(B, h, dtype=torch.bfloat16, device=dev)
        self.h = torch.zeros(B, h, dtype=torch.bfloat16, device=dev)
        self.qkv = torch.zeros(B, (model.hl + 2 * model.kl) * c.head_dim, dtype=torch.bfloat16, device=dev)
        self.attn = torch.zeros(B, model.hl * c.head_dim, dtype=torch.bfloat16, device=dev)
        self.logits = torch.zeros(B, c.vocab // model.tp.size, dtype=torch.bfloat16, device=dev)  # this rank's slice
        # gemm_dk deferred-norm partial sums [parts, 64] (a tuple: shared as-is by row views)
        self.ssq = tuple(torch.zeros(512 * 64, dtype=torch.float32, device=dev) for _ in range(2))
        self.temperature, self.seed, self.eos = temperature, seed, tuple(eos)[:4]
        self.graph = None

    def rows(self, b: int) -> "DecodeState":
        """A state over the first ``b`` rows of this one (views of the same buffers, its own graph):
        a decode step on it advances rows [0, b) exactly as the full state would, at batch-b cost."""
        v = object.__new__(DecodeState)
        for k, t in self.__dict__.items():
            v.__dict__[k] = t[:b] if isinstance(t, torch.Tensor) else t
        v.B, v.graph = b, None
        return v


def pack_prompts(prompts: list[list[int]]):
    lens = np.fromiter((len(p) for p in prompts), dtype=np.int64, count=len(prompts))
    cu = np.zeros(len(prompts) + 1, dtype=np.int32)
    np.cumsum(lens, out=cu[1:])
    flat = np.fromiter((t for p in prompts for t in p), dtype=np.int32, count=int(cu[-1]))
    pos = (np.arange(int(cu[-1]), dtype=np.int64) - np.repeat(cu[:-1], lens)).astype(np.int32)
    return flat, pos, cu, lens
