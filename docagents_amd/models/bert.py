"""BERT-family sentence encoder (BGE / E5) on the gfx950 kernels.

Replaces the OpenAI embeddings client (internal/embeddings/openai.go:38-127):
packed variable-length batches (no padding), fused embeddings+LayerNorm, GEMMs with fused
bias / GELU / residual epilogues, bidirectional varlen flash attention, and CLS (BGE) or mean (E5)
pooling fused with the L2 normalisation. Output vectors are unit-norm like the reference's
``normalize`` (openai.go:146-158).
"""
from __future__ import annotations

import math

import numpy as np
import torch

from ..ops import get_ops, h2d
from .configs import EncoderConfig

EPI_BIAS, EPI_GELU, EPI_RESID = 1, 2, 4


def _randn(shape, gen, device, std=0.02, dtype=torch.bfloat16):
    t = torch.empty(shape, dtype=torch.float32, device=device)
    t.normal_(0.0, std, generator=gen)
    return t.to(dtype)


class BertEncoder:
    """``dtype="fp8"``: the QKV and FFN-up projections run on e4m3 operands (SURVEY.md §7.2 step 7,
    BASELINE config 5 "fp8 MFMA embeddings"): weights quantised once per output channel, the
    LayerNorm kernels emit the per-token-quantised activations next to the bf16 rows, and the
    dequantisation is fused into the GEMM epilogue. Attention, the O / FFN-down projections
    (whose inputs would need a separate quantisation pass), pooling and the residual stream
    stay bf16.

    ``dtype="fp16"`` (BASELINE config 4 "BGE-large fp16 embedder"): every weight, activation and
    the residual stream in fp16 — GEMMs on v_mfma_f32_16x16x32_f16, flash attention on the 32x32x16
    f16 MFMA, fp16 LayerNorm / embeddings; fp32 accumulation; the pooled unit vectors come out fp32
    (and bf16 for the index, its storage type)."""

    LINEAR = ("wqkv", "w1")

    def __init__(self, cfg: EncoderConfig, device="cuda", seed: int = 0, weights: dict | None = None,
                 dtype: str = "bf16"):
        if dtype not in ("bf16", "fp8", "fp16"):
            raise ValueError(f"encoder dtype must be bf16, fp16 or fp8, got {dtype!r}")
        self.cfg = cfg
        self.device = torch.device(device)
        self.ops = get_ops(self.device)
        self.w = weights if weights is not None else self._random_init(seed)
        self.fp8 = dtype == "fp8"
        self.fp16 = dtype == "fp16"
        if self.fp16:  # one-time cast of the whole parameter set (an fp16 checkpoint loads as is)
            self.w = {k: (v.to(torch.float16) if isinstance(v, torch.Tensor) else
                          [{n: t.to(torch.float16) for n, t in L.items()} for L in v]) for k, v in self.w.items()}
        if self.fp8:
            for L in self.w["layers"]:
                for n in self.LINEAR:
                    L[n + "_q"], L[n + "_s"] = self.ops.quant_weight_fp8(L[n])
        import threading
        self._g_lock = threading.Lock()  # encode_one: the captured graphs' static buffers
        self._g_done = None              # event: the last graph use's output copied out

    def _linear(self, x, L, name, bias, epi, resid=None, xq=None):
        """fp8 path: ``xq = (q, scale)`` when the producer (a LayerNorm) already emitted the
        quantised rows; otherwise the layer stays bf16 (a standalone quantisation pass would cost
        more than the fp8 MFMA saves at these K, profiles/fp8_gemm_r1.txt)."""
        o = self.ops
        if xq is not None:
            return o.gemm_fp8(xq[0], xq[1], L[name + "_q"], L[name + "_s"], bias=bias, epi=epi, resid=resid)
        return o.gemm(x, L[name], bias=bias, epi=epi, resid=resid)

    # ------------------------------------------------------------------ weights
    def _random_init(self, seed: int) -> dict:
        c, dev = self.cfg, self.device
        gen = torch.Generator(device=dev)
        gen.manual_seed(seed * 7919 + 17)
        h, f = c.hidden, c.ffn
        ones = lambda n: torch.ones(n, dtype=torch.bfloat16, device=dev)  # noqa: E731
        zeros = lambda n: torch.zeros(n, dtype=torch.bfloat16, device=dev)  # noqa: E731
        w = {
            "word": _randn((c.vocab, h), gen, dev), "pos": _randn((c.max_pos, h), gen, dev),
            "type": _randn((c.type_vocab, h), gen, dev), "emb_ln_g": ones(h), "emb_ln_b": zeros(h),
            "layers": [],
        }
        for _ in range(c.layers):
            w["layers"].append({
                "wqkv": _randn((3 * h, h), gen, dev), "bqkv": zeros(3 * h),
                "wo": _randn((h, h), gen, dev), "bo": zeros(h),
                "ln1_g": ones(h), "ln1_b": zeros(h),
                "w1": _randn((f, h), gen, dev), "b1": zeros(f),
                "w2": _randn((h, f), gen, dev), "b2": zeros(h),
                "ln2_g": ones(h), "ln2_b": zeros(h),
            })
        return w

    @classmethod
    def from_hf_state_dict(cls, cfg: EncoderConfig, sd: dict, device="cuda", dtype: str = "bf16"):
        """Map a HF BertModel state dict (e.g. BGE safetensors) onto our packed layout."""
        dev = torch.device(device)
        g = lambda k: sd[k].to(device=dev, dtype=torch.bfloat16).contiguous()  # noqa: E731
        pre = "bert." if any(k.startswith("bert.") for k in sd) else ""
        w = {"word": g(pre + "embeddings.word_embeddings.weight"), "pos": g(pre + "embeddings.position_embeddings.weight"),
             "type": g(pre + "embeddings.token_type_embeddings.weight"),
             "emb_ln_g": g(pre + "embeddings.LayerNorm.weight"), "emb_ln_b": g(pre + "embeddings.LayerNorm.bias"),
             "layers": []}
        for i in range(cfg.layers):
            p = f"{pre}encoder.layer.{i}."
            w["layers"].append({
                "wqkv": torch.cat([g(p + f"attention.self.{n}.weight") for n in ("query", "key", "value")]).contiguous(),
                "bqkv": torch.cat([g(p + f"attention.self.{n}.bias") for n in ("query", "key", "value")]).contiguous(),
                "wo": g(p + "attention.output.dense.weight"), "bo": g(p + "attention.output.dense.bias"),
                "ln1_g": g(p + "attention.output.LayerNorm.weight"), "ln1_b": g(p + "attention.output.LayerNorm.bias"),
                "w1": g(p + "intermediate.dense.weight"), "b1": g(p + "intermediate.dense.bias"),
                "w2": g(p + "output.dense.weight"), "b2": g(p + "output.dense.bias"),
                "ln2_g": g(p + "output.LayerNorm.weight"), "ln2_b": g(p + "output.LayerNorm.bias"),
            })
        return cls(cfg, device, weights=w, dtype=dtype)

    # ------------------------------------------------------------------ forward
    def forward(self, ids: torch.Tensor, positions: torch.Tensor, cu_seqlens: torch.Tensor, max_seqlen: int):
        """ids/positions int32 [T] (packed), cu_seqlens int32 [B+1] -> hidden bf16 [T, H] (fp16 with
        dtype="fp16")."""
        c, o, w = self.cfg, self.ops, self.w
        if self.fp16:
            return self._forward_f16(ids, positions, cu_seqlens, max_seqlen)
        h, nh, hd = c.hidden, c.heads, c.head_dim
        q8 = self.fp8
        xq = None
        x = o.bert_embed_ln(ids, positions, None, w["word"], w["pos"], w["type"], w["emb_ln_g"], w["emb_ln_b"], c.eps,
                            fp8_out=q8)
        if q8:
            x, *xq = x
        for L in w["layers"]:
            qkv = self._linear(x, L, "wqkv", L["bqkv"], EPI_BIAS, xq=xq)
            a = o.flash_attn_varlen(qkv[:, :h], qkv[:, h:2 * h], qkv[:, 2 * h:], cu_seqlens, max_seqlen, nh, nh, hd,
                                    causal=False)
            x1 = self._linear(a, L, "wo", L["bo"], EPI_RESID, resid=x)
            x = o.layernorm(x1, L["ln1_g"], L["ln1_b"], c.eps, fp8_out=q8)
            if q8:
                x, *xq = x
            f = self._linear(x, L, "w1", L["b1"], EPI_GELU, xq=xq)
            x2 = self._linear(f, L, "w2", L["b2"], EPI_RESID, resid=x)
            x = o.layernorm(x2, L["ln2_g"], L["ln2_b"], c.eps, fp8_out=q8)
            if q8:
                x, *xq = x
        return x

    def _forward_f16(self, ids, positions, cu_seqlens, max_seqlen):
        c, o, w = self.cfg, self.ops, self.w
        h, nh, hd = c.hidden, c.heads, c.head_dim
        x = o.bert_embed_ln_f16(ids, positions, None, w["word"], w["pos"], w["type"], w["emb_ln_g"], w["emb_ln_b"],
                                c.eps)
        for L in w["layers"]:
            qkv = o.gemm_f16(x, L["wqkv"], bias=L["bqkv"], epi=EPI_BIAS)
            a = o.flash_attn_f16(qkv[:, :h], qkv[:, h:2 * h], qkv[:, 2 * h:], cu_seqlens, max_seqlen, nh, nh, hd)
            x1 = o.gemm_f16(a, L["wo"], bias=L["bo"], epi=EPI_RESID, resid=x)
            x = o.layernorm_f16(x1, L["ln1_g"], L["ln1_b"], c.eps)
            f = o.gemm_f16(x, L["w1"], bias=L["b1"], epi=EPI_GELU)
            x2 = o.gemm_f16(f, L["w2"], bias=L["b2"], epi=EPI_RESID, resid=x)
            x = o.layernorm_f16(x2, L["ln2_g"], L["ln2_b"], c.eps)
        return x

    def encode_packed(self, seqs: list[list[int]], out16: torch.Tensor | None = None) -> torch.Tensor:
        """Token-id sequences -> unit-norm embeddings. Returns bf16 [B, H] if out16 given else fp32."""
        lens = np.fromiter((len(s) for s in seqs), dtype=np.int64, count=len(seqs))
        if len(seqs) == 0:
            return torch.empty((0, self.cfg.hidden), dtype=torch.float32, device=self.device)
        cu = np.zeros(len(seqs) + 1, dtype=np.int32)
        np.cumsum(lens, out=cu[1:])
        flat = np.fromiter((t for s in seqs for t in s), dtype=np.int32, count=int(cu[-1]))
        pos = np.arange(int(cu[-1]), dtype=np.int32) - np.repeat(cu[:-1], lens)
        dev = self.device
        ids_t, pos_t, cu_t = h2d(flat, dev), h2d(pos, dev), h2d(cu, dev)
        hid = self.forward(ids_t, pos_t, cu_t, int(lens.max()))
        mode = 0 if self.cfg.pooling == "cls" else 1
        pool = self.ops.pool_l2norm_f16 if self.fp16 else self.ops.pool_l2norm
        if out16 is not None:
            return pool(hid, cu_t, mode, out16=out16)
        return pool(hid, cu_t, mode)

    # ---- one short sequence (a question) through captured HIP graphs ---------------------------
    # The eager encoder is ~90 launches, each paying its host-side launch path (~20 us from Python):
    # ~1.7 ms for a 20-token question, most of the p50 query's embed phase. One graph per padded
    # length bucket replays them in one submission. The rows past the real length are padding: the
    # GEMMs / norms process them (their rows are independent) and flash attention and the pooling
    # read the real length from cu_seqlens, so row 0..L-1 see exactly the unpadded computation.
    GRAPH_BUCKETS = (16, 32, 64, 128)
    # small batches of short texts (the fast embed lane's micro-batches of questions): one graph per
    # (sequences, padded tokens) bucket; sequences packed back to back, then padding rows, padded
    # sequences of length 0 (cu repeats the real total); every real length <= BATCH_MAX_LEN, which is
    # the max_seqlen the graphs were captured with. Measured: a lane batch took ~5 ms of launches
    # from Python beside the decode thread (profiles/r6/stack: es_embed)
    BATCH_BUCKETS = ((2, 64), (4, 128), (8, 256), (16, 512), (32, 1024), (64, 2048))
    BATCH_MAX_LEN = 128

    def _capture_small(self):
        from ..ops import kernels as K
        self._g, self._gb = {}, {}
        dev = self.device
        mode = 0 if self.cfg.pooling == "cls" else 1
        pool = self.ops.pool_l2norm_f16 if self.fp16 else self.ops.pool_l2norm
        side = torch.cuda.Stream(device=dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        Lc = self.BATCH_MAX_LEN
        # (key, T, max_seqlen, cu): the one-sequence length buckets and the batch buckets
        shapes = [(("one", T), T, T, [0, T]) for T in self.GRAPH_BUCKETS]
        for nb, T in self.BATCH_BUCKETS:
            step = min(Lc, (T - 1) // nb)
            shapes.append((("batch", nb), T, Lc, [i * step for i in range(nb + 1)]))
        bufs = {}
        # In a workspace role of their own, and EVERY shape warmed before the first capture: the
        # split-K scratch only grows, and a growth after a capture would free the memory that graph
        # captured (an illegal address at its next replay). The scratch is checked unchanged below.
        with torch.cuda.stream(side), K.workspace_role("enc_graph"):
            for key, T, ms, cu_l in shapes:
                ids = torch.zeros(T, dtype=torch.int32, device=dev)
                pos = torch.arange(T, dtype=torch.int32, device=dev) if key[0] == "one" else \
                    torch.zeros(T, dtype=torch.int32, device=dev)
                cu = torch.tensor(cu_l, dtype=torch.int32, device=dev)
                for _ in range(2):  # warm: allocations and workspaces before any capture
                    pool(self.forward(ids, pos, cu, ms), cu, mode)
                bufs[key] = (T, ms, ids, pos, cu)
            side.synchronize()
            ws0 = K.workspace_buffer(dev)
            for key, (T, ms, ids, pos, cu) in sorted(bufs.items(), key=lambda kv: -kv[1][0]):
                g = torch.cuda.CUDAGraph()
                # thread_local: a capture must not trip over the serving threads' own CUDA calls
                with torch.cuda.graph(g, stream=side, capture_error_mode="thread_local"):
                    out = pool(self.forward(ids, pos, cu, ms), cu, mode)
                if key[0] == "one":
                    self._g[T] = (g, ids, cu, out)
                else:
                    self._gb[key[1]] = (T, g, ids, pos, cu, out)
            if K.workspace_buffer(dev) is not ws0:
                raise RuntimeError("encoder graph capture grew the enc_graph workspace")
        torch.cuda.current_stream(dev).wait_stream(side)

    def prepare_graphs(self) -> None:
        """Capture the length-bucket graphs now (the engine does it at startup, before serving). A
        capture that fails leaves the eager path in charge (``_g`` empty), loudly."""
        if self.device.type == "cuda" and getattr(self, "_g", None) is None:
            try:
                self._capture_small()
            except Exception as e:  # noqa: BLE001 - the eager encoder still serves
                import logging
                logging.getLogger(__name__).warning("encoder graph capture failed, eager path: %r", e)
                self._g, self._gb = {}, {}

    def encode_one(self, seq: list[int]) -> torch.Tensor:
        """One token sequence -> unit-norm embedding fp32 [1, H]: a captured graph when it fits a
        length bucket on a GPU, else the eager packed path."""
        L = len(seq)
        if self.device.type != "cuda" or L == 0 or L > min(self.GRAPH_BUCKETS[-1], self.cfg.max_pos) or \
                torch.cuda.is_current_stream_capturing():
            return self.encode_packed([seq])
        if getattr(self, "_g", None) is None:
            self.prepare_graphs()
        T = next(b for b in self.GRAPH_BUCKETS if b >= L)
        if T not in self._g:
            return self.encode_packed([seq])
        g, ids, cu, out = self._g[T]
        host = torch.zeros(T + 2, dtype=torch.int32)
        host[:L] = torch.tensor(seq, dtype=torch.int32)
        host[T + 1] = L
        # The graphs' static buffers (ids / cu / out and the enc_graph workspace) are shared by every
        # caller, and callers run on streams of their own (the fast embed lane, the GPU thread).
        # Host order is not device order: each use waits on the device for the previous use's
        # clone (event chain) before its copies overwrite the inputs.
        with self._g_lock:
            cur = torch.cuda.current_stream(self.device)
            if self._g_done is not None:
                cur.wait_event(self._g_done)
            dev = h2d(host.numpy(), self.device)
            ids.copy_(dev[:T])
            cu.copy_(dev[T:])
            g.replay()
            res = out.clone()
            if self._g_done is None:
                self._g_done = torch.cuda.Event()
            self._g_done.record(cur)
        return res

    def encode_batch(self, seqs: list[list[int]]) -> torch.Tensor | None:
        """2..64 short sequences -> unit-norm embeddings fp32 [n, H] through a captured batch
        graph, or None when they fit no bucket (the caller runs the eager packed path)."""
        n = len(seqs)
        if self.device.type != "cuda" or n < 2 or torch.cuda.is_current_stream_capturing():
            return None
        if getattr(self, "_g", None) is None:
            self.prepare_graphs()
        lens = [len(q) for q in seqs]
        tot = sum(lens)
        if min(lens) == 0 or max(lens) > min(self.BATCH_MAX_LEN, self.cfg.max_pos):
            return None
        b = next((nb for nb, T in self.BATCH_BUCKETS if nb >= n and T > tot and nb in getattr(self, "_gb", {})), None)
        if b is None:
            return None
        T, g, ids, pos, cu, out = self._gb[b]
        host = np.zeros(2 * T + b + 1, dtype=np.int32)
        host[:tot] = np.fromiter((t for q in seqs for t in q), dtype=np.int32, count=tot)
        c = np.zeros(n + 1, dtype=np.int64)
        np.cumsum(lens, out=c[1:])
        host[T:T + tot] = np.arange(tot) - np.repeat(c[:-1], lens)
        host[2 * T:2 * T + n + 1] = c
        host[2 * T + n + 1:] = tot  # padded sequences: length 0
        with self._g_lock:  # the same device-side ordering as encode_one (shared workspace)
            cur = torch.cuda.current_stream(self.device)
            if self._g_done is not None:
                cur.wait_event(self._g_done)
            d = h2d(host, self.device)
            ids.copy_(d[:T])
            pos.copy_(d[T:2 * T])
            cu.copy_(d[2 * T:])
            g.replay()
            res = out[:n].clone()
            if self._g_done is None:
                self._g_done = torch.cuda.Event()
            self._g_done.record(cur)
        return res

    def flops_per_token(self, seqlen: int) -> float:
        c = self.cfg
        lin = 2 * (4 * c.hidden * c.hidden + 2 * c.hidden * c.ffn)
        return c.layers * (lin + 4 * seqlen * c.hidden)

    def param_bytes(self) -> int:
        return 2 * self.cfg.param_count()  # bf16 and fp16 alike


def pack_for_encoder(tok, texts: list[str], max_len: int, stats: dict | None = None) -> list[list[int]]:
    """Tokenize with [CLS]/[SEP] and truncate to the encoder's max positions (BERT max 512,
    SURVEY.md §5.7). Truncations are counted in ``stats`` (embed_truncated_texts / _tokens): a
    400-word enriched chunk can exceed 512 WordPiece tokens."""
    encs = tok.encode_batch(texts, add_special_tokens=True)
    out = []
    for e in encs:
        ids = e.ids
        if len(ids) > max_len:
            if stats is not None:
                stats["embed_truncated_texts"] = stats.get("embed_truncated_texts", 0) + 1
                stats["embed_truncated_tokens"] = stats.get("embed_truncated_tokens", 0) + len(ids) - max_len
            ids = ids[:max_len - 1] + [ids[-1]]
        out.append(ids)
    return out


def est_tokens(texts: list[str]) -> int:
    return int(math.fsum(len(t) for t in texts) / 4) + 2 * len(texts)
