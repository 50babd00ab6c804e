"""Plain-PyTorch fp32 reference implementations of every kernel in ``kernels.py``.

Used as the numerics oracle in tests (HIP kernel vs fp32 PyTorch of the same op) and as the
CPU execution path of the models (the container running CPU tests has no GPU). They are NOT a
GPU fallback: on a GPU device the models always call the HIP kernels.
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as F

EPI_NONE, EPI_BIAS, EPI_GELU, EPI_SWIGLU, EPI_RESID = 0, 1, 2, 3, 4
EPI_ROPE = 6  # gemm8p only: QKV + RoPE + KV-cache write


def gemv_fusable(M, N, K, epi=EPI_NONE):
    return M == 1


def gemm(a, w, bias=None, epi=EPI_NONE, resid=None, out=None, rms=None, **_):
    if rms is not None:  # same numerics as rmsnorm() followed by gemm() (bf16 normalised row)
        g = rms[0] if rms[0] is not None else torch.ones(a.shape[1], dtype=a.dtype, device=a.device)
        a = rmsnorm(a, g, rms[1])
    return _epilogue(a.float() @ w.float().t(), w.shape[0], bias, epi, resid, out)


def _epilogue(y, N, bias, epi, resid, out):
    if bias is not None:
        y = y + bias.float()
    if epi == EPI_GELU:
        y = F.gelu(y)
    elif epi == EPI_SWIGLU:
        yy = y.view(y.shape[0], N // 32, 2, 16)
        g, u = yy[:, :, 0, :], yy[:, :, 1, :]
        y = (F.silu(g) * u).reshape(y.shape[0], N // 2)
    elif epi == EPI_RESID:
        y = y + resid.float()
    y = y.to(torch.bfloat16)
    if out is not None:
        out.copy_(y)
        return out
    return y


def gemm_f16(a, w, bias=None, epi=EPI_NONE, resid=None, out=None):
    """fp16 oracle of kernels.gemm_f16: fp32 product + epilogue, one fp16 rounding."""
    y = a.float() @ w.float().t()
    if bias is not None:
        y = y + bias.float()
    if epi == EPI_GELU:
        y = F.gelu(y)
    elif epi == EPI_RESID:
        y = y + resid.float()
    y = y.to(torch.float16)
    if out is not None:
        out.copy_(y)
        return out
    return y


def interleave_gate_up(gate: torch.Tensor, up: torch.Tensor) -> torch.Tensor:
    """[F, K] gate + [F, K] up -> [2F, K] rows interleaved in 16-row groups (EPI_SWIGLU layout)."""
    Fd, K = gate.shape
    assert Fd % 16 == 0
    g = gate.view(Fd // 16, 16, K)
    u = up.view(Fd // 16, 16, K)
    return torch.stack([g, u], dim=1).reshape(2 * Fd, K).contiguous()


def rmsnorm(x, w, eps, resid=None, out=None):
    xf = x.float()
    if resid is not None:
        xf = xf + resid.float()
        resid.copy_(xf.to(resid.dtype))
    y = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps) * w.float()
    y = y.to(x.dtype)
    if out is not None:
        out.copy_(y)
        return out
    return y


def layernorm(x, g, b, eps, resid=None, out=None, fp8_out=False):
    xf = x.float()
    if resid is not None:
        xf = xf + resid.float()
    yf = F.layer_norm(xf, (xf.shape[-1],), g.float(), None if b is None else b.float(), eps)
    y = yf.to(x.dtype)
    if out is not None:
        out.copy_(y)
        y = out
    if fp8_out:
        yq, ys = quant_fp8(yf)
        return y, yq, ys
    return y


def bert_embed_ln(ids, positions, types, word, pos, type_, g, b, eps, out=None, fp8_out=False):
    t = type_[types.long()] if types is not None else type_[0]
    x = word[ids.long()].float() + pos[positions.long()].float() + t.float()
    return layernorm(x.to(word.dtype), g, b, eps, out=out, fp8_out=fp8_out)


def embed(ids, table, out=None):
    y = table[ids.long()]
    if out is not None:
        out.copy_(y)
        return out
    return y


def pool_l2norm(h, cu_seqlens, mode=0, out32=None, out16=None):
    cu = cu_seqlens.tolist()
    rows = []
    for i in range(len(cu) - 1):
        s0, s1 = cu[i], cu[i + 1]
        if mode == 0 or s1 <= s0:
            rows.append(h[s0].float())
        else:
            rows.append(h[s0:s1].float().mean(0))
    v = torch.stack(rows) if rows else torch.zeros((0, h.shape[1]))
    n = v.norm(dim=-1, keepdim=True)
    v = torch.where(n > 0, v / n.clamp_min(1e-30), v)
    if out16 is not None:
        out16.copy_(v.to(out16.dtype))
    if out32 is not None:
        out32.copy_(v)
        return out32
    return v if out16 is None else out16


def rope_table(max_pos: int, D: int, theta: float, device=None) -> torch.Tensor:
    inv = 1.0 / (theta ** (torch.arange(0, D, 2, dtype=torch.float64) / D))
    t = torch.arange(max_pos, dtype=torch.float64)
    ang = torch.outer(t, inv)
    return torch.stack([ang.cos(), ang.sin()], dim=-1).float().contiguous().to(device)


def _rope_rows(x, cs):  # x [T, nh, D], cs [T, D/2, 2]; pairs (2i, 2i+1) rotated by theta_i * pos
    x1, x2 = x[..., 0::2].float(), x[..., 1::2].float()
    c, s = cs[:, None, :, 0], cs[:, None, :, 1]
    return torch.stack([x1 * c - x2 * s, x2 * c + x1 * s], dim=-1).flatten(-2)


def gemm_rope(a, w, pos, cos_sin, H, Hkv, D, slot, k_cache, v_cache, out=None, kv_out=True):
    """QKV projection with RoPE on q / k and the k / v cache write fused (gemm + rope_cache)."""
    qkv = gemm(a, w, out=out)
    return rope_cache(qkv, pos, cos_sin, H, Hkv, D, slot=slot, k_cache=k_cache, v_cache=v_cache)


def rope_cache(qkv, pos, cos_sin, H, Hkv, D, slot=None, k_cache=None, v_cache=None, rotate_q=True):
    T = qkv.shape[0]
    x = qkv.view(T, H + 2 * Hkv, D)
    cs = cos_sin[pos.long()]
    if rotate_q:
        x[:, :H] = _rope_rows(x[:, :H], cs).to(qkv.dtype)
    x[:, H:H + Hkv] = _rope_rows(x[:, H:H + Hkv], cs).to(qkv.dtype)
    if k_cache is not None:
        sl, ps = slot.long(), pos.long()
        k_cache[sl, :, ps] = x[:, H:H + Hkv]
        v_cache[sl, :, ps] = x[:, H + Hkv:]
    return qkv


def flash_kv_cache_ok(D: int, causal: bool) -> bool:
    return causal


def flash_attn_varlen(q, k, v, cu_seqlens, max_seqlen, H, Hkv, D, causal, scale=None, out=None, prefix=None,
                      kv_cache=None):
    """prefix = (k_pre [Hkv, >=P, D], v_pre, P): every sequence's keys are the P shared prefix keys
    followed by its own; query i sits at key position P + i (bottom-right causal).
    kv_cache = (k_cache, v_cache, slot, pos): own keys of the sequence starting at token t read from
    k_cache[slot[t], :, pos[t] + j] (k / v ignored)."""
    if kv_cache is not None:
        kc, vc, ks, kpos = kv_cache
        T = q.shape[0]
        cu = cu_seqlens.tolist()
        k = torch.empty((T, Hkv * D), dtype=q.dtype, device=q.device)
        v = torch.empty((T, Hkv * D), dtype=q.dtype, device=q.device)
        for b in range(len(cu) - 1):
            s0, s1 = cu[b], cu[b + 1]
            if s1 > s0:
                sl, p0 = int(ks[s0]), int(kpos[s0])
                k[s0:s1] = kc[sl, :, p0:p0 + s1 - s0].transpose(0, 1).reshape(s1 - s0, Hkv * D)
                v[s0:s1] = vc[sl, :, p0:p0 + s1 - s0].transpose(0, 1).reshape(s1 - s0, Hkv * D)
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    T = q.shape[0]
    res = torch.empty((T, H * D), dtype=q.dtype, device=q.device)
    cu = cu_seqlens.tolist()
    G = H // Hkv
    P = 0 if prefix is None else int(prefix[2])
    if P:
        kp = prefix[0][:, :P].float().repeat_interleave(G, 0)   # [H, P, D]
        vp = prefix[1][:, :P].float().repeat_interleave(G, 0)
    for b in range(len(cu) - 1):
        s0, s1 = cu[b], cu[b + 1]
        L = s1 - s0
        if L == 0:
            continue
        qq = q[s0:s1, :H * D].float().view(L, H, D).transpose(0, 1)
        kk = k[s0:s1, :Hkv * D].float().view(L, Hkv, D).transpose(0, 1).repeat_interleave(G, 0)
        vv = v[s0:s1, :Hkv * D].float().view(L, Hkv, D).transpose(0, 1).repeat_interleave(G, 0)
        if P:
            kk, vv = torch.cat([kp, kk], 1), torch.cat([vp, vv], 1)
        s = (qq @ kk.transpose(1, 2)) * scale
        if causal:
            m = torch.ones(L, P + L, dtype=torch.bool, device=q.device).triu(P + 1)
            s = s.masked_fill(m, float("-inf"))
        p = s.softmax(-1)
        res[s0:s1] = (p @ vv).transpose(0, 1).reshape(L, H * D).to(q.dtype)
    if out is not None:
        out.copy_(res)
        return out
    return res


def decode_attn(q, k_cache, v_cache, lens, slot, H, Hkv, D, max_len=None, chunk=256, scale=None, out=None, pre=None,
                rope=None):
    """pre: optional int32 [B, 2] = (P, prefix slot): keys [0, P) of row b come from the prefix slot.
    rope = (cos_sin, pos): q is the raw qkv row; RoPE + the new token's cache write happen here
    (rope_cache on a copy of the rows, then attention)."""
    if rope is not None:
        q = rope_cache(q.clone(), rope[1], rope[0], H, Hkv, D, slot=slot, k_cache=k_cache, v_cache=v_cache)
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    B = q.shape[0]
    G = H // Hkv
    res = torch.empty((B, H * D), dtype=q.dtype, device=q.device)
    pre_h = None if pre is None else pre.tolist()
    for b in range(B):
        L, s = int(lens[b]), int(slot[b])
        qq = q[b, :H * D].float().view(H, 1, D)
        kk = k_cache[s, :, :L].float()
        vv = v_cache[s, :, :L].float()
        if pre_h is not None and pre_h[b][0] > 0:
            P, ps = pre_h[b]
            kk = torch.cat([k_cache[ps, :, :P].float(), kk[:, P:]], 1)
            vv = torch.cat([v_cache[ps, :, :P].float(), vv[:, P:]], 1)
        kk, vv = kk.repeat_interleave(G, 0), vv.repeat_interleave(G, 0)
        p = ((qq @ kk.transpose(1, 2)) * scale).softmax(-1)
        res[b] = (p @ vv).reshape(H * D).to(q.dtype)
    if out is not None:
        out.copy_(res)
        return out
    return res


def log_softmax_rows(logits):
    return torch.log_softmax(logits.float(), dim=-1)


_M32 = 0xFFFFFFFF


def _hash_u32(x: np.ndarray) -> np.ndarray:
    """common.h hash_u32 on uint32 arrays (numpy uint32 arithmetic wraps mod 2^32, like the kernel)."""
    x = x ^ (x >> np.uint32(16))
    x = x * np.uint32(0x7feb352d)
    x = x ^ (x >> np.uint32(15))
    x = x * np.uint32(0x846ca68b)
    return x ^ (x >> np.uint32(16))


def gumbel_u01(seed: int, rkey, v) -> np.ndarray:
    """The sampler kernel's counter-based uniform (common.h u01(seed, rkey, v)), bit-exact; rkey and
    v broadcast (uint32-valued integer arrays)."""
    with np.errstate(over="ignore"):
        rk = np.asarray(rkey, dtype=np.uint32)
        vv = np.asarray(v, dtype=np.uint32)
        inner = _hash_u32(vv + np.uint32(0x632be5ab))
        h = _hash_u32(np.uint32(seed & _M32) ^ _hash_u32(rk + np.uint32(0x9e3779b9) * inner))
    return ((h >> np.uint32(8)).astype(np.float64) + 0.5) * (1.0 / 16777216.0)


def _gumbel_scores(x, temperature, seed, rkeys, v0=0):
    """x fp32 [B, V] -> Gumbel-max scores x / T - log(-log u(seed, rkey_b, v0 + v)) (T <= 0: x)."""
    if temperature <= 0:
        return x.double()
    B, V = x.shape
    u = gumbel_u01(seed, rkeys.reshape(B, 1), np.arange(v0, v0 + V, dtype=np.int64).reshape(1, V))
    return x.double().cpu() / temperature - torch.from_numpy(np.log(-np.log(u)))


def _rkeys(B, step, ctr) -> np.ndarray:
    rs = (ctr.cpu().numpy()[:B].astype(np.int64) if ctr is not None else np.full(B, step, dtype=np.int64))
    with np.errstate(over="ignore"):
        return rs.astype(np.uint32) * np.uint32(131071) + np.arange(B, dtype=np.uint32)


def _bookkeep(B, tok, chosen, device, out_tok=None, out_lp=None, conf=None, active=None, pos=None, lens=None,
              hist=None, start=None, eos=()):
    on = active.bool().clone() if active is not None else torch.ones(B, dtype=torch.bool, device=device)
    if out_tok is None:
        out_tok = torch.zeros(B, dtype=torch.int32, device=device)
    out_tok.copy_(torch.where(on, tok, out_tok))
    if out_lp is not None:
        out_lp.copy_(torch.where(on, chosen, out_lp))
    if conf is not None:
        conf[:, 0] += torch.where(on, chosen.exp(), torch.zeros_like(chosen))
        conf[:, 1] += on.float()
    stop = torch.zeros(B, dtype=torch.bool, device=device)
    for e in list(eos)[:4]:
        stop |= tok == e
    if hist is not None:
        gi = (pos - start).long()
        for b in range(B):
            if on[b] and 0 <= gi[b] < hist.shape[1]:
                hist[b, gi[b]] = tok[b]
        stop |= (gi + 1) >= hist.shape[1]
    if pos is not None:
        pos += on.int()
    if lens is not None:
        lens += on.int()
    if active is not None:
        active.copy_(torch.where(on & stop, torch.zeros_like(active), active))
    return out_tok, chosen


def sample(logits, temperature, seed, step=0, out_tok=None, out_lp=None, conf=None, active=None, ctr=None,
           pos=None, lens=None, hist=None, start=None, eos=()):
    """Reference sampler with the kernel's semantics: Gumbel-max at temperature T with the kernel's
    counter-based hash noise (greedy when T <= 0; ties to the lower index), the chosen token's
    log-probability under the untempered distribution, and the device-side bookkeeping."""
    B = logits.shape[0]
    lp = log_softmax_rows(logits)
    sc = _gumbel_scores(logits.float().cpu(), temperature, seed, _rkeys(B, step, ctr))
    tok = sc.argmax(-1).to(logits.device)  # first maximal index = the kernel's lower-index tie rule
    chosen = lp.gather(1, tok.view(-1, 1)).squeeze(1)
    return _bookkeep(B, tok.int(), chosen, logits.device, out_tok, out_lp, conf, active, pos, lens, hist, start, eos)


def sample_partial(logits, temperature, seed, v0, step=0, ctr=None, out=None):
    """Vocab-parallel sampling, rank side (see ops.kernels.sample_partial): stats fp32 [B, 8]."""
    B, V = logits.shape
    x = logits.float().cpu()
    sc = _gumbel_scores(x, temperature, seed, _rkeys(B, step, ctr), v0)
    bi = sc.argmax(-1)
    mx = x.max(-1).values
    st = torch.zeros((B, 8), dtype=torch.float32)
    st[:, 0] = sc.gather(1, bi.view(-1, 1)).squeeze(1).float()
    st[:, 1] = (bi + v0).to(torch.int32).view(torch.float32)
    st[:, 2] = mx
    st[:, 3] = torch.exp(x - mx[:, None]).sum(-1)
    st[:, 4] = x.gather(1, bi.view(-1, 1)).squeeze(1)
    st = st.to(logits.device)
    if out is not None:
        out.copy_(st)
        return out
    return st


def sample_finalize(gathered, ranks, out_tok=None, out_lp=None, conf=None, active=None, pos=None, lens=None,
                    hist=None, start=None, eos=()):
    """Vocab-parallel sampling, merge side: gathered [B, ranks * 8] -> sample()'s outputs."""
    B = gathered.shape[0]
    g = gathered.float().cpu().view(B, ranks, 8)
    score, idx = g[..., 0], g[..., 1].contiguous().view(torch.int32).long()
    best = score.max(-1).values
    cand = torch.where(score == best[:, None], idx, torch.full_like(idx, 1 << 40))
    r = cand.argmin(-1)  # max score, ties to the lower global index
    tok = idx.gather(1, r.view(-1, 1)).squeeze(1)
    xb = g[..., 4].gather(1, r.view(-1, 1)).squeeze(1).double()
    gmax = g[..., 2].max(-1).values.double()
    lse = gmax + torch.log((g[..., 3].double() * torch.exp(g[..., 2].double() - gmax[:, None])).sum(-1))
    chosen = (xb - lse).float().to(gathered.device)
    return _bookkeep(B, tok.int().to(gathered.device), chosen, gathered.device, out_tok, out_lp, conf, active, pos,
                     lens, hist, start, eos)


def topk_dense(X, Qv, K, thr, slots=None, bitmap=None, **_):
    s = Qv.float() @ X.float().t()  # [Q, N]
    valid = s >= thr
    if slots is not None:
        valid &= (slots[:X.shape[0]] >= 0).view(1, -1)
    if bitmap is not None:
        sl = slots[:X.shape[0]].long().clamp_min(0)
        words = bitmap[:, (sl >> 5)]  # [Q, N]
        bits = (words >> (sl & 31).view(1, -1)) & 1
        valid &= bits.bool()
    s = s.masked_fill(~valid, float("-inf"))
    return _topk_with_ties(s, K)


def _topk_with_ties(s, K):
    Q, N = s.shape
    if N == 0:
        return (torch.full((Q, K), float("-inf")), torch.full((Q, K), -1, dtype=torch.int32))
    # sort desc by score, asc by index
    idx = torch.arange(N, device=s.device).expand(Q, N)
    order = torch.argsort(idx, dim=1, stable=True)
    vals, perm = torch.sort(s, dim=1, descending=True, stable=True)
    ids = torch.gather(idx, 1, perm)
    kk = min(K, N)
    vs, ii = vals[:, :kk], ids[:, :kk].int()
    ii = torch.where(torch.isinf(vs), torch.full_like(ii, -1), ii)
    if kk < K:
        vs = torch.cat([vs, torch.full((Q, K - kk), float("-inf"), device=s.device)], 1)
        ii = torch.cat([ii, torch.full((Q, K - kk), -1, dtype=torch.int32, device=s.device)], 1)
    del order
    return vs, ii


def topk_ranges(X, Qv, ranges, range_off, K, thr, max_rows=None, slots=None, bitmap=None, **_):
    Q = Qv.shape[0]
    N = X.shape[0]
    s = Qv.float() @ X.float().t()
    allowed = torch.zeros((Q, N), dtype=torch.bool, device=X.device)
    ro = range_off.tolist()
    rg = ranges.tolist()
    for q in range(Q):
        for r in range(ro[q], ro[q + 1]):
            a, b = rg[r]
            allowed[q, a:b] = True
    valid = allowed & (s >= thr)
    if slots is not None:
        valid &= (slots[:N] >= 0).view(1, -1)
    if bitmap is not None:
        sl = slots[:N].long().clamp_min(0)
        bits = (bitmap[:, (sl >> 5)] >> (sl & 31).view(1, -1)) & 1
        valid &= bits.bool()
    s = s.masked_fill(~valid, float("-inf"))
    return _topk_with_ties(s, K)


def topk_merge(cand_s, cand_i, K):
    P, Q, _ = cand_s.shape
    s = cand_s.permute(1, 0, 2).reshape(Q, -1)
    i = cand_i.permute(1, 0, 2).reshape(Q, -1)
    s = torch.where(i < 0, torch.full_like(s, float("-inf")), s)
    # sort by score desc, id asc
    big = i.clamp_min(0).to(torch.float64)
    key = s.to(torch.float64) * 1e12 - big
    order = torch.argsort(key, dim=1, descending=True, stable=True)
    vs, ii = torch.gather(s, 1, order)[:, :K], torch.gather(i, 1, order)[:, :K]
    ii = torch.where(torch.isinf(vs), torch.full_like(ii, -1), ii)
    return vs, ii


def kmeans_accum(X, assign, sums, counts):
    a = assign.long()
    m = a >= 0
    sums.index_add_(0, a[m], X[m].float())
    counts.index_add_(0, a[m], torch.ones(int(m.sum()), device=X.device))


# ----------------------------------------------------------------------------------- fp8 path
def quant_fp8(x, out=None, scale=None):
    xf = x.float()
    sc = xf.abs().amax(dim=1) / 448.0
    sc = torch.where(sc > 0, sc, torch.ones_like(sc))
    q = (xf / sc[:, None]).clamp(-448, 448).to(torch.float8_e4m3fn)
    if out is not None:
        out.copy_(q)
        q = out
    if scale is not None:
        scale[:sc.numel()].copy_(sc)
        sc = scale
    return q, sc


def gemm_fp8(aq, sa, wq, sw, bias=None, epi=EPI_NONE, resid=None, out=None):
    y = (aq.float() * sa[:aq.shape[0], None].float()) @ (wq.float() * sw[:, None].float()).t()
    return _epilogue(y, wq.shape[0], bias, epi, resid, out)


def quant_weight_fp8(w):
    wf = w.float()
    sw = (wf.abs().amax(dim=1) / 448.0).clamp_min(1e-30)
    return (wf / sw[:, None]).clamp(-448, 448).to(torch.float8_e4m3fn).contiguous(), sw.contiguous()


DECODE_DK = True
# above 32 rows the split-K tiles stay faster (bench/midm_chain.py, profiles/r3/dk/): the narrow
# dk tiles re-read the activation block once per 16-64 weight rows
DK_MAX_M = 64
DK_SPLITK_ABOVE = 32


def dk_fusable(M, N, K, epi=EPI_NONE):
    return (DECODE_DK and 2 <= M <= DK_MAX_M and K % 256 == 0 and N % 16 == 0
            and epi in (EPI_NONE, EPI_BIAS, EPI_RESID, EPI_SWIGLU) and (epi != EPI_SWIGLU or N % 32 == 0))


def dk_parts(N, M=0):
    """gemm_dk.hip dk_bn for EPI_RESID: row-norm partial sums written per output tile; 33..64 rows
    (the split-K route): one per 512 columns (written by the reduce launch)."""
    if DK_SPLITK_ABOVE < M <= 64 and N % 512 == 0:
        return N // 512
    bn = 64 if N // 64 >= 192 else (32 if N // 32 >= 192 else 16)
    return (N + bn - 1) // bn


def gemm_dk(a, w, epi=EPI_NONE, bias=None, resid=None, out=None, norm_in=None, ssq_out=None):
    """gemm_dk.hip: optional deferred row RMSNorm of ``a`` from partial sums of squares, then the
    product + epilogue; EPI_RESID may also emit the new rows' per-part sums of squares."""
    M, K = a.shape
    N = w.shape[0]
    x = a.float()
    if norm_in is not None:
        ssq, parts, eps = norm_in
        inv = torch.rsqrt(ssq.view(-1, 64)[:parts, :M].sum(0) / K + eps)
        x = (x * inv[:, None]).to(torch.bfloat16).float()
    y = _epilogue(x @ w.float().t(), N, bias, epi, resid, out)
    if ssq_out is not None:
        parts = dk_parts(N, M)
        bn = -(-N // parts)
        y2 = y.float().pow(2)
        sq = torch.stack([y2[:, i * bn:(i + 1) * bn].sum(-1) for i in range(parts)])  # [parts, M]
        ssq_out.view(-1, 64)[:parts, :M] = sq
    return y


def gemm_resid_norm(a, w, resid, gamma, eps, out=None, h_out=None, bias=None):
    y = gemm(a, w, bias=bias, epi=EPI_RESID, resid=resid)
    (resid if out is None else out).copy_(y)
    h = rmsnorm(y, gamma, eps)
    if h_out is not None:
        h_out.copy_(h)
        return h_out
    return h


# fp16 forms of the encoder ops (kernels.*_f16): these references keep the input dtype
layernorm_f16 = layernorm
bert_embed_ln_f16 = bert_embed_ln
pool_l2norm_f16 = pool_l2norm


def flash_attn_f16(q, k, v, cu_seqlens, max_seqlen, H, Hkv, D, causal=False, scale=None, out=None):
    y = flash_attn_varlen(q.float(), k.float(), v.float(), cu_seqlens, max_seqlen, H, Hkv, D, causal, scale=scale)
    y = y.to(torch.float16)
    if out is not None:
        out.copy_(y)
        return out
    return y
