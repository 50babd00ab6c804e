"""Numerics of every gfx950 HIP kernel vs the plain-PyTorch fp32 reference of the same op."""

import numpy as np

import pytest
import torch

pytestmark = pytest.mark.gpu

from docagents_amd.ops import kernels as K  # noqa: E402
from docagents_amd.ops import reference as R  # noqa: E402

DEV = "cuda"


def _rand(*shape, scale=1.0, dtype=torch.bfloat16):
    return (torch.randn(*shape, device=DEV) * scale).to(dtype)


def _close(a, b, atol, rtol=0.02):
    a, b = a.float(), b.float()
    err = (a - b).abs()
    tol = atol + rtol * b.abs()
    bad = (err > tol).sum().item()
    assert bad == 0, f"{bad} / {a.numel()} mismatches, max err {err.max().item():.4g}"


@pytest.mark.parametrize("M,N,Kd", [(1, 128, 64), (7, 200, 128), (33, 256, 192), (64, 384, 256),
                                    (130, 264, 320), (257, 1024, 768), (512, 768, 3072)])
@pytest.mark.parametrize("epi", [K.EPI_NONE, K.EPI_BIAS, K.EPI_GELU, K.EPI_RESID])
def test_gemm(M, N, Kd, epi):
    torch.manual_seed(M * 1000 + N)
    a, w = _rand(M, Kd), _rand(N, Kd, scale=Kd ** -0.5)
    bias = _rand(N) if epi != K.EPI_NONE else None
    resid = _rand(M, N) if epi == K.EPI_RESID else None
    got = K.gemm(a, w, bias=bias, epi=epi, resid=resid)
    ref = R.gemm(a, w, bias=bias, epi=epi, resid=resid)
    _close(got, ref, atol=0.03)


@pytest.mark.parametrize("tile", [1, 2, 3])
@pytest.mark.parametrize("splits", [1, 2, 4])
def test_gemm_tiles_splitk(tile, splits):
    torch.manual_seed(tile * 10 + splits)
    M, N, Kd = 96, 512, 512
    a, w, bias = _rand(M, Kd), _rand(N, Kd, scale=Kd ** -0.5), _rand(N)
    got = K.gemm(a, w, bias=bias, epi=K.EPI_BIAS, tile=tile, splits=splits)
    _close(got, R.gemm(a, w, bias=bias, epi=K.EPI_BIAS), atol=0.03)


@pytest.mark.parametrize("M,F,splits", [(5, 256, 1), (64, 512, 2), (300, 1024, 1), (40, 2048, 4)])
def test_gemm_swiglu(M, F, splits):
    torch.manual_seed(M)
    Kd = 256
    gate, up = _rand(F, Kd, scale=Kd ** -0.5), _rand(F, Kd, scale=Kd ** -0.5)
    w = R.interleave_gate_up(gate, up)
    a = _rand(M, Kd)
    got = K.gemm(a, w, epi=K.EPI_SWIGLU, splits=splits)
    ref = (torch.nn.functional.silu(a.float() @ gate.float().t()) * (a.float() @ up.float().t()))
    _close(got, ref, atol=0.03)


@pytest.mark.parametrize("M,N,Kd", [(256, 256, 128), (300, 520, 192), (1000, 1032, 768), (2048, 3072, 3072),
                                    (129, 264, 640), (4100, 776, 256)])
@pytest.mark.parametrize("epi", [K.EPI_NONE, K.EPI_BIAS, K.EPI_GELU, K.EPI_RESID, K.EPI_SWIGLU])
@pytest.mark.parametrize("tile", [7, 10])
def test_gemm8p_tile(M, N, Kd, epi, tile):
    """Phase-split kernel, 256-row (tile 7) and 128-row (tile 10) tiles, every epilogue, ragged M / N."""
    torch.manual_seed(M + N + epi)
    if epi == K.EPI_SWIGLU:
        N = (N // 32) * 32
    a, w = _rand(M, Kd), _rand(N, Kd, scale=Kd ** -0.5)
    bias = _rand(N) if epi in (K.EPI_BIAS, K.EPI_GELU, K.EPI_RESID) else None
    resid = _rand(M, N) if epi == K.EPI_RESID else None
    got = K.gemm(a, w, bias=bias, epi=epi, resid=resid, tile=tile, splits=1)
    ref = R.gemm(a, w, bias=bias, epi=epi, resid=resid)
    _close(got, ref, atol=0.04)


@pytest.mark.parametrize("M,N,Kd", [(256, 256, 128), (300, 520, 192), (1000, 1032, 768), (2048, 3072, 3072),
                                    (129, 264, 640), (4100, 776, 256), (777, 2048, 1024)])
@pytest.mark.parametrize("epi", [K.EPI_NONE, K.EPI_BIAS, K.EPI_GELU, K.EPI_RESID, K.EPI_SWIGLU])
def test_gemm4w_tile(M, N, Kd, epi):
    """Four-wave 256x256 kernel (tile 13, the A/B arm of csrc/gemm4w.hip; asm MFMAs with AGPR
    accumulators): its schedules (three fragment sets with two / one barriers per K-tile at K / 64
    even >= 4, two sets otherwise or forced) on every epilogue and ragged M / N vs the fp32
    reference, and bit-identical to each other (same MFMA order per accumulator)."""
    torch.manual_seed(M + N + epi + 13)
    if epi == K.EPI_SWIGLU:
        N = (N // 32) * 32
    a, w = _rand(M, Kd), _rand(N, Kd, scale=Kd ** -0.5)
    bias = _rand(N) if epi in (K.EPI_BIAS, K.EPI_GELU, K.EPI_RESID) else None
    resid = _rand(M, N) if epi == K.EPI_RESID else None
    prev = K.gemm4w_variant(0)
    try:
        got = K.gemm(a, w, bias=bias, epi=epi, resid=resid, tile=13, splits=1)
        others = []
        for v in (1, 2):
            K.gemm4w_variant(v)
            others.append(K.gemm(a, w, bias=bias, epi=epi, resid=resid, tile=13, splits=1))
    finally:
        K.gemm4w_variant(prev)
    _close(got, R.gemm(a, w, bias=bias, epi=epi, resid=resid), atol=0.04)
    for o in others:
        assert torch.equal(got, o)


@pytest.mark.parametrize("M,N,Kd", [(4100, 4104, 256), (2304, 9216, 192), (3000, 9216, 128), (2600, 3072, 3072)])
@pytest.mark.parametrize("epi", [K.EPI_NONE, K.EPI_BIAS, K.EPI_GELU, K.EPI_RESID, K.EPI_SWIGLU])
@pytest.mark.parametrize("tile", [7, 10])
def test_gemm8p_persistent(M, N, Kd, epi, tile):
    """More tiles than CUs: the persistent tile loop (workgroups running 1-3 tiles each, ragged M / N;
    K = 128 / 192 / 256 / 3072: every K-loop shape of the first K-tile whose counted waits let the
    previous tile's stores fly) vs the fp32 reference, and bit-identical to one workgroup per tile."""
    torch.manual_seed(M + N + epi + tile)
    if epi == K.EPI_SWIGLU:
        N = (N // 32) * 32
    a, w = _rand(M, Kd), _rand(N, Kd, scale=Kd ** -0.5)
    bias = _rand(N) if epi in (K.EPI_BIAS, K.EPI_GELU, K.EPI_RESID) else None
    resid = _rand(M, N) if epi == K.EPI_RESID else None
    prev = K.gemm8p_persist(1)
    try:
        got = K.gemm(a, w, bias=bias, epi=epi, resid=resid, tile=tile, splits=1)
        K.gemm8p_persist(0)
        one = K.gemm(a, w, bias=bias, epi=epi, resid=resid, tile=tile, splits=1)
    finally:
        K.gemm8p_persist(prev)
    _close(got, R.gemm(a, w, bias=bias, epi=epi, resid=resid), atol=0.04)
    assert torch.equal(got, one)


@pytest.mark.parametrize("M", [256, 700, 3000])
@pytest.mark.parametrize("H,Hkv,D", [(32, 32, 96), (8, 2, 128), (4, 4, 64)])
def test_gemm_rope(M, H, Hkv, D):
    """QKV projection with RoPE + KV-cache write in the GEMM epilogue == gemm + rope_cache (fp32 ref),
    and bit-identical to the in-tree gemm -> rope_cache kernels."""
    torch.manual_seed(M + D)
    Kd = 256
    N = (H + 2 * Hkv) * D
    a, w = _rand(M, Kd), _rand(N, Kd, scale=Kd ** -0.5)
    S, L = 5, 1024
    slot = torch.randint(0, S, (M,), device=DEV, dtype=torch.int32)
    pos = torch.randperm(L, device=DEV)[:M].to(torch.int32) if M <= L else \
        torch.arange(M, device=DEV, dtype=torch.int32) % L
    if M > L:  # keep (slot, pos) unique
        slot = (torch.arange(M, device=DEV, dtype=torch.int32) // L).to(torch.int32)
        S = int(slot.max()) + 1
    cs = R.rope_table(L, D, 10000.0, device=DEV)
    kc = torch.zeros(S, Hkv, L, D, device=DEV, dtype=torch.bfloat16)
    vc = torch.zeros_like(kc)
    kc2, vc2, kc3, vc3 = kc.clone(), vc.clone(), kc.clone(), vc.clone()
    got = K.gemm_rope(a, w, pos, cs, H, Hkv, D, slot, kc, vc)
    ref = R.gemm_rope(a, w, pos, cs, H, Hkv, D, slot, kc2, vc2)
    _close(got, ref, atol=0.03)
    _close(kc, kc2, atol=0.03)
    _close(vc, vc2, atol=0.03)
    two = K.rope_cache(K.gemm(a, w), pos, cs, H, Hkv, D, slot=slot, k_cache=kc3, v_cache=vc3)
    assert torch.equal(got, two) and torch.equal(kc, kc3) and torch.equal(vc, vc3)


@pytest.mark.parametrize("M", [65, 128, 200])
def test_gemm_mid_m_in_tree(M):
    """65..255 rows with split-K (auto): the 128x64 weight-streaming tile to 128 rows, the 64x128 tile
    over ceil(M/64) row blocks above; plain / SwiGLU / residual epilogues, vs the fp32 reference."""
    torch.manual_seed(M)
    N, F, Kd = 3072, 1024, 3072
    a, w = _rand(M, Kd), _rand(N, Kd, scale=Kd ** -0.5)
    assert K._auto_splits(M, N, Kd) > 1
    ref = a.float() @ w.float().t()
    _close(K.gemm(a, w), ref, atol=0.03)
    resid = _rand(M, N)
    x = resid.clone()
    K.gemm(a, w, epi=K.EPI_RESID, resid=x, out=x)
    _close(x, ref + resid.float(), atol=0.05)
    gate, up = _rand(F, Kd, scale=Kd ** -0.5), _rand(F, Kd, scale=Kd ** -0.5)
    got = K.gemm(a, R.interleave_gate_up(gate, up), epi=K.EPI_SWIGLU)
    _close(got, torch.nn.functional.silu(a.float() @ gate.float().t()) * (a.float() @ up.float().t()), atol=0.03)


def test_gemm_strided_a():
    big = _rand(50, 3 * 256)
    a = big[:, 256:512]
    w = _rand(128, 256, scale=1 / 16)
    _close(K.gemm(a, w), R.gemm(a.contiguous(), w), atol=0.03)


@pytest.mark.parametrize("D", [768, 3072, 4096])
def test_rmsnorm(D):
    x, w = _rand(37, D), _rand(D)
    r1 = _rand(37, D)
    r2 = r1.clone()
    got = K.rmsnorm(x, w, 1e-5, resid=r1)
    ref = R.rmsnorm(x, w, 1e-5, resid=r2)
    _close(got, ref, atol=0.02)
    _close(r1, r2, atol=0.01)
    _close(K.rmsnorm(x, w, 1e-5), R.rmsnorm(x, w, 1e-5), atol=0.02)


@pytest.mark.parametrize("D", [2048, 3072, 4096, 2560])
def test_rmsnorm_many_rows(D):
    """>= 1024 rows of a width made of whole 512-element slices take the one-wave-per-row kernel
    (2560: not a supported slice count, the per-row workgroup kernel); both vs the fp32 reference,
    with and without the fused residual add, and row-strided input / output."""
    M = 1500
    x, w = _rand(M, D + 64)[:, :D], _rand(D)
    r1 = _rand(M, D)
    r2 = r1.clone()
    got = K.rmsnorm(x, w, 1e-5, resid=r1)
    _close(got, R.rmsnorm(x, w, 1e-5, resid=r2), atol=0.02)
    _close(r1, r2, atol=0.01)
    out = torch.zeros(M, D + 128, device=DEV, dtype=torch.bfloat16)
    K.rmsnorm(x, w, 1e-5, out=out[:, :D])
    _close(out[:, :D], R.rmsnorm(x, w, 1e-5), atol=0.02)
    assert float(out[:, D:].abs().max()) == 0.0


@pytest.mark.parametrize("D", [384, 768, 1024])
def test_layernorm_and_embed(D):
    x, g, b = _rand(19, D), _rand(D), _rand(D)
    _close(K.layernorm(x, g, b, 1e-12), R.layernorm(x, g, b, 1e-12), atol=0.03)
    res = _rand(19, D)
    _close(K.layernorm(x, g, b, 1e-12, resid=res), R.layernorm(x, g, b, 1e-12, resid=res), atol=0.03)
    word, pos, typ = _rand(100, D), _rand(64, D), _rand(2, D)
    ids = torch.randint(0, 100, (23,), device=DEV, dtype=torch.int32)
    ps = torch.randint(0, 64, (23,), device=DEV, dtype=torch.int32)
    _close(K.bert_embed_ln(ids, ps, None, word, pos, typ, g, b, 1e-12),
           R.bert_embed_ln(ids, ps, None, word, pos, typ, g, b, 1e-12), atol=0.03)
    _close(K.embed(ids, word), R.embed(ids, word), atol=0)


@pytest.mark.parametrize("mode", [0, 1])
def test_pool_l2norm(mode):
    h = _rand(50, 768)
    cu = torch.tensor([0, 5, 5, 20, 50], device=DEV, dtype=torch.int32)
    got = K.pool_l2norm(h, cu, mode)
    ref = R.pool_l2norm(h, cu, mode)
    _close(got, ref, atol=2e-3)
    n = got.norm(dim=-1)
    assert torch.allclose(n, torch.ones_like(n), atol=1e-3)


@pytest.mark.parametrize("H,Hkv,D", [(4, 4, 96), (8, 2, 128), (4, 1, 64)])
def test_rope_cache(H, Hkv, D):
    T = 21
    qkv = _rand(T, (H + 2 * Hkv) * D)
    pos = torch.randint(0, 100, (T,), device=DEV, dtype=torch.int32)
    slot = torch.randint(0, 3, (T,), device=DEV, dtype=torch.int32)
    pos = pos + torch.arange(T, device=DEV, dtype=torch.int32) * 0  # distinct writes not required
    # make (slot, pos) unique so cache writes are deterministic
    pos = torch.arange(T, device=DEV, dtype=torch.int32) * 3
    cs = R.rope_table(128, D, 10000.0, device=DEV)
    kc1 = torch.zeros(3, Hkv, 128, D, device=DEV, dtype=torch.bfloat16)
    vc1 = torch.zeros_like(kc1)
    kc2, vc2 = kc1.clone(), vc1.clone()
    a, b = qkv.clone(), qkv.clone()
    K.rope_cache(a, pos, cs, H, Hkv, D, slot=slot, k_cache=kc1, v_cache=vc1)
    R.rope_cache(b, pos, cs, H, Hkv, D, slot=slot, k_cache=kc2, v_cache=vc2)
    _close(a, b, atol=0.02)
    _close(kc1, kc2, atol=0.02)
    _close(vc1, vc2, atol=0)


@pytest.mark.parametrize("D", [32, 64, 96, 128])
@pytest.mark.parametrize("causal,H,Hkv", [(False, 4, 4), (True, 8, 2), (True, 4, 4)])
def test_flash_attn(D, causal, H, Hkv):
    torch.manual_seed(D + H)
    lens = [1, 63, 64, 65, 200, 7]
    cu = torch.tensor([0] + list(torch.tensor(lens).cumsum(0)), device=DEV, dtype=torch.int32)
    T = sum(lens)
    qkv = _rand(T, (H + 2 * Hkv) * D)
    q = qkv[:, :H * D]
    k = qkv[:, H * D:(H + Hkv) * D]
    v = qkv[:, (H + Hkv) * D:]
    got = K.flash_attn_varlen(q, k, v, cu, max(lens), H, Hkv, D, causal)
    ref = R.flash_attn_varlen(q, k, v, cu, max(lens), H, Hkv, D, causal)
    _close(got, ref, atol=0.02)


@pytest.mark.parametrize("D", [64, 96])
def test_flash_attn_spike(D):
    # force a late rescale: one key dominates one query (online-softmax branch coverage; causal D = 96
    # runs the speculative softmax of the pipelined kernel: the deferred-max branch, whose overshoot
    # threshold it exceeds)
    H, Hkv = 2, 2
    L = 300
    qkv = _rand(L, 6 * D, scale=0.3)
    qkv[250, 2 * D:3 * D] = 4.0
    qkv[10, :D] = 4.0
    cu = torch.tensor([0, L], device=DEV, dtype=torch.int32)
    q, k, v = qkv[:, :2 * D], qkv[:, 2 * D:4 * D], qkv[:, 4 * D:]
    for causal in (False, True):
        _close(K.flash_attn_varlen(q, k, v, cu, L, H, Hkv, D, causal),
               R.flash_attn_varlen(q, k, v, cu, L, H, Hkv, D, causal), atol=0.02)


@pytest.mark.parametrize("D", [64, 96, 128])
@pytest.mark.parametrize("lens,chunk", [([1000], 512), ([1], 256), ([513, 257, 64], 256), ([2944] * 5, 0),
                                        ([65, 1024, 700], 64), ([2935], 0), ([1000, 3], 768),
                                        ([300] * 9 + [1, 2000], 0), ([4000, 64, 129] * 4, 512)])
def test_decode_attn_fused_rope(D, lens, chunk):
    """Decode attention with RoPE + the new token's cache write folded in == rope_cache + attention,
    on the small-batch (prefetching, B * Hkv <= 32) and the streaming (larger batches) variants."""
    torch.manual_seed(D + len(lens) + chunk)
    B = len(lens)
    H, slots, max_seq = 4, B + 2, 4096
    kc, vc = _rand(slots, H, max_seq, D), _rand(slots, H, max_seq, D)
    qkv = _rand(B, 3 * H * D)
    L = torch.tensor(lens, dtype=torch.int32, device=DEV)
    pos = L - 1
    slot = torch.arange(B, dtype=torch.int32, device=DEV) + 1
    cs = R.rope_table(max_seq, D, 10000.0, device=DEV)
    kc2, vc2, qkv2, qkv0 = kc.clone(), vc.clone(), qkv.clone(), qkv.clone()
    K.rope_cache(qkv2, pos, cs, H, H, D, slot=slot, k_cache=kc2, v_cache=vc2)
    want = K.decode_attn(qkv2, kc2, vc2, L, slot, H, H, D, max_seq, chunk=chunk)
    got = K.decode_attn(qkv, kc, vc, L, slot, H, H, D, max_seq, chunk=chunk, rope=(cs, pos))
    _close(got, want, atol=0.01)
    for b in range(B):
        s_, p_ = int(slot[b]), int(pos[b])
        _close(kc[s_, :, p_], kc2[s_, :, p_], atol=0.01)
        assert torch.equal(vc[s_, :, p_], vc2[s_, :, p_])
    assert torch.equal(qkv, qkv0)  # q / k rows untouched (the kernel rotates on the fly)
    ref = R.decode_attn(qkv.clone(), kc.clone(), vc.clone(), L, slot, H, H, D, rope=(cs, pos))
    _close(got, ref, atol=0.02)


@pytest.mark.parametrize("D", [64, 96, 128])
@pytest.mark.parametrize("B,chunk", [(1, 512), (2, 256), (3, 1024), (1, 64)])
def test_decode_attn_prefetch_variant(D, B, chunk):
    """MHA decode with the next tile prefetched (B rows alone: B * Hkv <= 32) == the streaming variant
    (the same rows inside a batch padded past 32 (row, kv head) pairs)."""
    torch.manual_seed(D + B)
    H, slots, max_seq = 8, 4, 2048
    kc, vc = _rand(slots, H, max_seq, D), _rand(slots, H, max_seq, D)
    q = _rand(B, H * D)
    lens = torch.tensor([1000, 1537, 63][:B], dtype=torch.int32, device=DEV)
    slot = torch.tensor([2, 0, 3][:B], dtype=torch.int32, device=DEV)
    pad = 8  # B + 8 rows x 8 heads > 32 pairs: the streaming variant
    qp = torch.cat([q, _rand(pad, H * D)])
    lp = torch.cat([lens, torch.full((pad,), 100, dtype=torch.int32, device=DEV)])
    sp = torch.cat([slot, torch.zeros(pad, dtype=torch.int32, device=DEV)])
    small = K.decode_attn(q, kc, vc, lens, slot, H, H, D, max_seq, chunk=chunk)
    big = K.decode_attn(qp, kc, vc, lp, sp, H, H, D, max_seq, chunk=chunk)[:B]
    ref = R.decode_attn(q, kc, vc, lens, slot, H, H, D, max_seq)
    _close(small, ref, atol=0.02)
    _close(small, big, atol=0.01)


@pytest.mark.parametrize("H,Hkv,D", [(32, 32, 96), (32, 8, 128), (8, 2, 64)])
@pytest.mark.parametrize("rope", [False, True])
def test_decode_attn_balanced_splits(H, Hkv, D, rope):
    """Balanced splits (a row's L keys spread over every split of the capacity-sized grid) match the
    fp32 reference, including rows shorter than one split and rows on a split boundary, with the
    in-kernel merge (fused RoPE: MHA only)."""
    if rope and H != Hkv:
        pytest.skip("fused RoPE decode is MHA only")
    torch.manual_seed(H + D + rope)
    max_seq = 4096
    lens_l = [2935, 1, 512, 4000, 63]
    B = len(lens_l)
    kc, vc = _rand(B + 2, Hkv, max_seq, D), _rand(B + 2, Hkv, max_seq, D)
    q = _rand(B, (H + 2 * Hkv) * D)
    lens = torch.tensor(lens_l, dtype=torch.int32, device=DEV)
    slot = torch.arange(B, dtype=torch.int32, device=DEV) + 1
    cs = R.rope_table(max_seq, D, 10000.0, device=DEV)
    rp = (cs, lens - 1) if rope else None
    ref = R.decode_attn(q.clone(), kc.clone(), vc.clone(), lens, slot, H, Hkv, D, rope=rp)
    got = K.decode_attn(q, kc.clone(), vc.clone(), lens, slot, H, Hkv, D, max_len=max_seq, chunk=512, rope=rp)
    _close(got, ref, atol=0.02)


def test_decode_xc_probe_round_robin():
    """The placement probe behind the same-XCD decode exchange: on an SPX MI355X a launch's workgroup w
    runs on XCD w % 8 (8 distinct XCC ids, one per residue)."""
    assert K.decode_xc_ok(torch.device(DEV))


@pytest.mark.parametrize("B,H,rope", [(1, 32, False), (1, 32, True), (2, 16, True), (4, 8, False)])
@pytest.mark.parametrize("lens0", [2937, 64, 1])
def test_decode_attn_same_xcd_exchange(B, H, rope, lens0, monkeypatch):
    """Splits merged through one XCD's L2 (cached partials + L2 ticket) == the uncached cross-XCD merge,
    bit for bit, and vs the fp32 reference; repeated launches (the counters must return to zero)."""
    torch.manual_seed(B * H + lens0)
    D, max_seq = 96, 4096
    kc, vc = _rand(B + 1, H, max_seq, D), _rand(B + 1, H, max_seq, D)
    q = _rand(B, 3 * H * D)
    lens = torch.tensor([lens0, 1500, 333, 4000][:B], dtype=torch.int32, device=DEV)
    slot = torch.arange(B, dtype=torch.int32, device=DEV) + 1
    cs = R.rope_table(max_seq, D, 10000.0, device=DEV)
    rp = (cs, lens - 1) if rope else None
    assert K.decode_xc_ok(torch.device(DEV)) and (B * H) % 8 == 0 and B * H <= 32
    outs = {}
    for xc in (True, False):
        monkeypatch.setattr(K, "DECODE_XC", xc)
        k2, v2 = kc.clone(), vc.clone()
        outs[xc] = [K.decode_attn(q, k2, v2, lens, slot, H, H, D, max_len=max_seq, rope=rp) for _ in range(3)]
        outs[xc].append((k2, v2))
    for i in range(3):
        assert torch.equal(outs[True][i], outs[False][i]) and torch.equal(outs[True][i], outs[True][0])
    assert torch.equal(outs[True][3][0], outs[False][3][0]) and torch.equal(outs[True][3][1], outs[False][3][1])
    ref = R.decode_attn(q.clone(), kc.clone(), vc.clone(), lens, slot, H, H, D, rope=rp)
    _close(outs[True][0], ref, atol=0.02)


@pytest.mark.parametrize("H,Hkv,D", [(32, 32, 96), (32, 8, 128), (8, 1, 128), (12, 6, 64)])
def test_decode_attn(H, Hkv, D):
    torch.manual_seed(H * D)
    B, S = 5, 700
    kc, vc = _rand(7, Hkv, S, D), _rand(7, Hkv, S, D)
    lens = torch.tensor([1, 64, 65, 300, 700], device=DEV, dtype=torch.int32)
    slot = torch.tensor([6, 0, 3, 2, 1], device=DEV, dtype=torch.int32)
    q = _rand(B, (H + 2 * Hkv) * D)
    got = K.decode_attn(q, kc, vc, lens, slot, H, Hkv, D, max_len=700, chunk=128)
    ref = R.decode_attn(q, kc, vc, lens, slot, H, Hkv, D)
    _close(got, ref, atol=0.02)


def test_sample_greedy_and_logprob():
    torch.manual_seed(0)
    B, V = 6, 32064
    logits = _rand(B, V, scale=3.0)
    conf = torch.zeros(B, 2, device=DEV)
    tok, lp = K.sample(logits, 0.0, 1, 0, conf=conf)
    rtok, rlp = R.sample(logits, 0.0, 1, 0)
    assert torch.equal(tok.cpu(), rtok.cpu())
    _close(lp, rlp, atol=2e-3)
    _close(conf[:, 0], rlp.exp(), atol=2e-3)
    assert torch.all(conf[:, 1] == 1)


def test_sample_temperature_distribution():
    # Gumbel-max with the hash RNG must follow softmax(logits / T)
    V = 8
    logits = torch.tensor([[0.0, 0.5, 1.0, 0.2, -1.0, 0.3, 0.1, 0.9]], device=DEV).to(torch.bfloat16)
    logits = logits.repeat(4096, 1).contiguous()
    tok, _ = K.sample(logits, 0.7, 1234, 5)
    counts = torch.bincount(tok.long().cpu(), minlength=V).float() / 4096
    p = torch.softmax(logits[0].float().cpu() / 0.7, -1)
    assert (counts - p).abs().max() < 0.03


def test_sample_kernel_rng_matches_reference():
    """The reference sampler reproduces the kernel's counter-based Gumbel noise (bit-exact uniforms;
    fp32 vs fp64 logs can only flip near-ties), so sampled tokens are comparable at T > 0 too."""
    torch.manual_seed(1)
    B, V = 64, 32064
    logits = _rand(B, V, scale=3.0)
    ctr = torch.arange(B, dtype=torch.int32, device=DEV) * 7 + 300
    tok, lp = K.sample(logits, 0.2, 4242, 0, ctr=ctr.clone())
    rtok, rlp = R.sample(logits, 0.2, 4242, 0, ctr=ctr.clone())
    assert (tok.cpu() == rtok.cpu()).float().mean() >= 0.95
    same = tok.cpu() == rtok.cpu()
    _close(lp.cpu()[same], rlp.cpu()[same], atol=2e-3)


@pytest.mark.parametrize("T", [0.0, 0.2, 1.0])
@pytest.mark.parametrize("B,V", [(1, 32064), (3, 32064), (8, 128256), (2, 5000), (64, 32064)])
def test_sample_chunked_matches_one_workgroup_per_row(T, B, V):
    """Small batches cut each row over ceil(V / 1024) workgroups + finalize (sample_chunk_kernel):
    the same tokens and bookkeeping as one workgroup per row (sample_kernel), logprobs to rounding,
    including a tie between chunks (the lower index wins)."""
    torch.manual_seed(B * 7 + V)
    logits = _rand(B, V, scale=3.0)
    logits[0, 17] = logits[0, V - 3] = 60.0

    def state():
        return dict(out_tok=torch.zeros(B, dtype=torch.int32, device=DEV), out_lp=torch.zeros(B, device=DEV),
                    conf=torch.zeros(B, 2, device=DEV),
                    active=(torch.arange(B, device=DEV) % 5 != 3).int(),
                    pos=torch.arange(B, dtype=torch.int32, device=DEV) + 40,
                    lens=torch.arange(B, dtype=torch.int32, device=DEV) + 41,
                    hist=torch.full((B, 8), -1, dtype=torch.int32, device=DEV),
                    start=torch.full((B,), 39, dtype=torch.int32, device=DEV))
    a, b = state(), state()
    old = K.SAMPLE_CHUNKED_MAX_B
    try:
        K.SAMPLE_CHUNKED_MAX_B = 0
        K.sample(logits, T, 99, 0, ctr=a["pos"], eos=(5,), **a)
        K.SAMPLE_CHUNKED_MAX_B = 64
        K.sample(logits, T, 99, 0, ctr=b["pos"], eos=(5,), **b)
    finally:
        K.SAMPLE_CHUNKED_MAX_B = old
    torch.cuda.synchronize()
    assert a["out_tok"][0].item() == 17 or T > 0
    for k in a:
        if k in ("out_lp", "conf"):
            _close(a[k], b[k], atol=1e-4)
        else:
            assert torch.equal(a[k], b[k]), k


@pytest.mark.parametrize("T", [0.0, 0.2, 1.0])
@pytest.mark.parametrize("ranks", [2, 8])
def test_sample_partial_finalize_matches_full_row(T, ranks):
    """Vocab-parallel sampling: per-slice 8-float summaries + finalize == the
    sampler on the full rows (tokens, logprobs, bookkeeping), including a tie across slices."""
    torch.manual_seed(ranks)
    B, V = 48, 128256
    Vl = V // ranks
    logits = _rand(B, V, scale=3.0)
    logits[0, 11] = logits[0, V - 2] = 60.0

    def state():
        return dict(out_tok=torch.zeros(B, dtype=torch.int32, device=DEV), out_lp=torch.zeros(B, device=DEV),
                    conf=torch.zeros(B, 2, device=DEV),
                    active=(torch.arange(B, device=DEV) % 7 != 3).int(),
                    pos=torch.arange(B, dtype=torch.int32, device=DEV) + 50,
                    lens=torch.arange(B, dtype=torch.int32, device=DEV) + 51,
                    hist=torch.full((B, 8), -1, dtype=torch.int32, device=DEV),
                    start=torch.full((B,), 49, dtype=torch.int32, device=DEV))
    a, b = state(), state()
    K.sample(logits, T, 77, 0, ctr=a["pos"], eos=(5,), **a)
    stats = torch.cat([K.sample_partial(logits[:, r * Vl:(r + 1) * Vl].contiguous(), T, 77, r * Vl, ctr=b["pos"])
                       for r in range(ranks)], dim=1).contiguous()
    K.sample_finalize(stats, ranks, eos=(5,), **b)
    torch.cuda.synchronize()
    for k in a:
        if k in ("out_lp", "conf"):
            _close(a[k], b[k], atol=1e-4)
        else:
            assert torch.equal(a[k], b[k]), k
    if T == 0.0:
        assert int(b["out_tok"][0]) == 11


@pytest.mark.parametrize("N,d,Q,Kk", [(1000, 768, 5, 5), (5000, 1024, 37, 20), (63, 768, 1, 3), (20000, 768, 16, 1),
                                      (300000, 1024, 64, 10), (7000, 384, 3, 32), (4000, 512, 8, 5),
                                      (3000, 768, 300, 4), (40000, 384, 100, 8), (2000, 768, 17, 3)])
def test_topk_dense(N, d, Q, Kk):
    """The streaming scans (d 384 / 768 / 1024: one query block per wave run up to 16 queries, four
    query blocks sharing LDS tiles above, up to 256 queries) and the query-major tiles (other d,
    k-means-sized batches) vs fp32: plain, filtered + floored, and with removed rows (slot -1)."""
    torch.manual_seed(N)
    X = torch.nn.functional.normalize(torch.randn(N, d, device=DEV), dim=-1).to(torch.bfloat16)
    Qv = torch.nn.functional.normalize(torch.randn(Q, d, device=DEV), dim=-1).to(torch.bfloat16)
    Qv[0] = X[N // 2]
    s, i = K.topk_dense(X, Qv, Kk, -1.0)
    rs, ri = R.topk_dense(X, Qv, Kk, -1.0)
    _close(s, rs, atol=2e-3)
    assert (i == ri).float().mean() > 0.97
    assert int(i[0, 0]) == N // 2
    # filter + threshold
    slots = (torch.arange(N, device=DEV, dtype=torch.int32) // 10).contiguous()
    W = (N // 10 + 32) // 32
    bitmap = torch.zeros(Q, W, dtype=torch.int32, device=DEV)
    bitmap[:, 0] = 0b1011
    bitmap[0, (N // 2 // 10) >> 5] |= (1 << ((N // 2 // 10) & 31))
    s, i = K.topk_dense(X, Qv, Kk, 0.0, slots=slots, bitmap=bitmap)
    rs, ri = R.topk_dense(X, Qv, Kk, 0.0, slots=slots, bitmap=bitmap)
    _close(s, rs, atol=2e-3)
    assert torch.equal(i.cpu(), ri.cpu()) or (s - rs).abs().max() < 2e-3
    # removed rows (slot -1) never match, including the query's own row
    slots2 = torch.zeros(N, dtype=torch.int32, device=DEV)
    slots2[N // 2] = -1
    slots2[::7] = -1
    s, i = K.topk_dense(X, Qv, Kk, -1.0, slots=slots2)
    rs, ri = R.topk_dense(X, Qv, Kk, -1.0, slots=slots2)
    _close(s, rs, atol=2e-3)
    assert not bool((i == N // 2).any()) and not bool(((i >= 0) & (i % 7 == 0)).any())


@pytest.mark.parametrize("Q", [3, 20, 64])
def test_topk_dense_ties(Q):
    """Exact score ties at the k-th place go to the smaller row id (the scans' radix-select cut and
    the merge): 50 copies of one row, queried with that row, must return its 8 smallest ids."""
    torch.manual_seed(Q)
    N, d, Kk = 20000, 1024, 8
    X = torch.nn.functional.normalize(torch.randn(N, d, device=DEV), dim=-1).to(torch.bfloat16)
    X[7000:7050] = X[7000]
    X[150:160] = X[7000]  # ten more copies in another row block, smaller ids
    Qv = torch.nn.functional.normalize(torch.randn(Q, d, device=DEV), dim=-1).to(torch.bfloat16)
    Qv[Q - 1] = X[7000]
    s, i = K.topk_dense(X, Qv, Kk, -1.0)
    assert i[Q - 1].tolist() == list(range(150, 158))
    assert bool((s[Q - 1] == s[Q - 1, 0]).all())
    rs, ri = R.topk_dense(X, Qv, Kk, -1.0)
    _close(s, rs, atol=2e-3)


def test_topk_ranges():
    torch.manual_seed(1)
    N, d, Q, Kk = 3000, 768, 4, 6
    X = torch.nn.functional.normalize(torch.randn(N, d, device=DEV), dim=-1).to(torch.bfloat16)
    Qv = torch.nn.functional.normalize(torch.randn(Q, d, device=DEV), dim=-1).to(torch.bfloat16)
    rg = [[0, 10], [100, 700], [2990, 3000], [5, 6], [0, 3000], [1000, 1001]]
    ro = [0, 3, 4, 5, 6]
    ranges = torch.tensor(rg, dtype=torch.int32, device=DEV)
    roff = torch.tensor(ro, dtype=torch.int32, device=DEV)
    s, i = K.topk_ranges(X, Qv, ranges, roff, Kk, -1.0, max_rows=3000, rows_per_split=256)
    rs, ri = R.topk_ranges(X, Qv, ranges, roff, Kk, -1.0)
    _close(s, rs, atol=2e-3)
    assert (i == ri).float().mean() > 0.95
    assert int(i[1, 0]) == 5 and int(i[1, 1]) == -1  # single-row range


def test_kmeans_accum():
    X = _rand(500, 256)
    assign = torch.randint(-1, 10, (500,), device=DEV, dtype=torch.int32)
    s1, c1 = torch.zeros(10, 256, device=DEV), torch.zeros(10, device=DEV)
    s2, c2 = s1.clone(), c1.clone()
    K.kmeans_accum(X, assign, s1, c1)
    R.kmeans_accum(X, assign, s2, c2)
    _close(s1, s2, atol=1e-3)
    assert torch.equal(c1, c2)


@pytest.mark.parametrize("H,Hkv,D", [(32, 8, 128), (8, 1, 128), (16, 8, 64), (8, 2, 96)])
def test_decode_attn_gqa(H, Hkv, D):
    """GQA decode: the MFMA kernel (D = 64 / 128) and the VALU kernel (other head dims) vs fp32."""
    torch.manual_seed(7)
    B, S = 4, 1500
    kc, vc = _rand(4, Hkv, S, D), _rand(4, Hkv, S, D)
    lens = torch.tensor([3, 129, 1000, 1500], device=DEV, dtype=torch.int32)
    slot = torch.tensor([3, 1, 0, 2], device=DEV, dtype=torch.int32)
    q = _rand(B, (H + 2 * Hkv) * D)
    a = K.decode_attn(q, kc, vc, lens, slot, H, Hkv, D, max_len=S)
    _close(a, R.decode_attn(q, kc, vc, lens, slot, H, Hkv, D), atol=0.02)


@pytest.mark.parametrize("M,N,Kd,epi", [(300, 768, 768, 0), (512, 3072, 768, 2), (1000, 768, 3072, 4),
                                         (256, 2304, 1024, 1)])
def test_gemm_fp8_matches_dequantized_reference(M, N, Kd, epi):
    torch.manual_seed(M + N)
    x = _rand(M, Kd)
    w = _rand(N, Kd, scale=Kd ** -0.5)
    bias = _rand(N) if epi in (1, 2, 4) else None
    resid = _rand(M, N) if epi == 4 else None
    xq, sa = K.quant_fp8(x)
    rq, rsa = R.quant_fp8(x)
    assert torch.allclose(sa, rsa, rtol=1e-6)
    # both round to nearest even; x*(1/s) vs x/s may land on opposite sides of a rounding boundary
    d = (xq.float() - rq.float()).abs()
    assert (d > 0).float().mean().item() < 1e-2
    assert torch.all(d <= 0.126 * rq.float().abs() + 2 ** -9)
    wq, sw = K.quant_weight_fp8(w)
    got = K.gemm_fp8(xq, sa, wq, sw, bias=bias, epi=epi, resid=resid)
    ref = R.gemm_fp8(xq, sa, wq, sw, bias=bias, epi=epi, resid=resid)
    _close(got, ref, atol=0.03)
    full = R.gemm(x, w, bias=bias, epi=epi, resid=resid)
    rel = (got.float() - full.float()).norm() / full.float().norm()
    assert rel < 0.06, rel


def test_encoder_fp8_vs_bf16_gpu():
    from docagents_amd.models.bert import BertEncoder
    from docagents_amd.models.configs import encoder_config
    cfg = encoder_config("bge-small")
    a = BertEncoder(cfg, DEV, seed=5)
    b = BertEncoder(cfg, DEV, weights=a.w, dtype="fp8")
    seqs = [[101] + list(range(1000, 1000 + n)) + [102] for n in (5, 60, 300)]
    cos = (a.encode_packed(seqs) * b.encode_packed(seqs)).sum(-1)
    assert torch.all(cos > 0.97), cos


def test_layernorm_fused_fp8_output():
    torch.manual_seed(11)
    x, r = _rand(333, 768), _rand(333, 768)
    g, b = _rand(768) + 1, _rand(768)
    y, yq, ys = K.layernorm(x, g, b, 1e-12, resid=r, fp8_out=True)
    ry, rq, rs = R.layernorm(x, g, b, 1e-12, resid=r, fp8_out=True)
    _close(y, ry, atol=0.03)
    assert torch.allclose(ys, rs, rtol=1e-3)
    d = (yq.float() * ys[:, None] - rq.float() * rs[:, None]).abs()
    assert torch.all(d <= 0.13 * (rq.float() * rs[:, None]).abs() + 1e-3)


@pytest.mark.parametrize("N,Kd", [(96, 512), (544, 3072), (1024, 8192), (32064, 3072), (256, 2560), (128, 4608)])
@pytest.mark.parametrize("epi", [K.EPI_NONE, K.EPI_BIAS, K.EPI_RESID, K.EPI_SWIGLU])
def test_gemv_batch1_decode(N, Kd, epi):
    torch.manual_seed(N + Kd + epi)
    if epi == K.EPI_SWIGLU:
        N = (N // 32) * 32
    a, w = _rand(1, Kd), _rand(N, Kd, scale=Kd ** -0.5)
    bias = _rand(N) if epi in (K.EPI_BIAS, K.EPI_RESID) else None
    resid = _rand(1, N) if epi == K.EPI_RESID else None
    got = K.gemm(a, w, bias=bias, epi=epi, resid=resid, tile=6, splits=1)
    ref = R.gemm(a, w, bias=bias, epi=epi, resid=resid)
    _close(got, ref, atol=0.03)
    auto = K.gemm(a, w, bias=bias, epi=epi, resid=resid)  # M = 1 auto-selects the GEMV
    assert torch.equal(auto, got)


@pytest.mark.parametrize("N,Kd", [(3072, 8192), (1000, 16384), (8, 8192), (3072, 9216)])
@pytest.mark.parametrize("epi", [K.EPI_NONE, K.EPI_BIAS, K.EPI_RESID])
def test_gemv_long_rows_two_waves(N, Kd, epi):
    """Batch-1 GEMV on narrow matrices with long rows (the K=8192 down projection): two waves split
    each row's K range and combine through LDS == fp32 (plain and with the RMSNorm fused)."""
    torch.manual_seed(N + Kd + epi)
    a, w = _rand(1, Kd), _rand(N, Kd, scale=Kd ** -0.5)
    bias = _rand(N) if epi in (K.EPI_BIAS, K.EPI_RESID) else None
    resid = _rand(1, N) if epi == K.EPI_RESID else None
    got = K.gemm(a, w, bias=bias, epi=epi, resid=resid, tile=6, splits=1)
    g = _rand(Kd) + 1.0
    x = _rand(1, Kd, scale=3.0)
    fused = K.gemm(x, w, epi=epi, bias=bias, resid=resid, rms=(g, 1e-5))
    _close(got, R.gemm(a, w, bias=bias, epi=epi, resid=resid), atol=0.03)
    _close(fused, R.gemm(x, w, bias=bias, epi=epi, resid=resid, rms=(g, 1e-5)), atol=0.03)


@pytest.mark.parametrize("N,Kd,epi", [(9216, 3072, K.EPI_NONE), (1024, 3072, K.EPI_SWIGLU), (32064, 3072, K.EPI_NONE)])
def test_gemv_fused_rmsnorm(N, Kd, epi):
    torch.manual_seed(N)
    x = _rand(1, Kd, scale=3.0)
    g = _rand(Kd) + 1.0
    w = _rand(N, Kd, scale=Kd ** -0.5)
    got = K.gemm(x, w, epi=epi, rms=(g, 1e-5))
    unfused = K.gemm(K.rmsnorm(x, g, 1e-5), w, epi=epi, tile=6, splits=1)
    _close(got, unfused, atol=0.03)
    _close(got, R.gemm(x, w, epi=epi, rms=(g, 1e-5)), atol=0.03)


@pytest.mark.parametrize("D,causal", [(64, False), (96, True), (128, True), (32, False), (64, True), (96, False),
                                      (128, False), (32, True)])
def test_flash_attn_dispatch_shapes(D, causal):
    """Every kernel the flash dispatch picks (the pipelined causal D = 96 kernel, the 4-wave and the
    8-wave D = 128 flash_attn_v2 shapes) against the fp32 reference, GQA, ragged lengths."""
    torch.manual_seed(D + causal)
    lens = [1, 77, 300, 513]
    H, Hkv = 4, 2
    T = sum(lens)
    q, k, v = _rand(T, H * D), _rand(T, Hkv * D), _rand(T, Hkv * D)
    cu = torch.tensor([0] + list(np.cumsum(lens)), device=DEV, dtype=torch.int32)
    got = K.flash_attn_varlen(q, k, v, cu, max(lens), H, Hkv, D, causal)
    _close(got, R.flash_attn_varlen(q, k, v, cu, max(lens), H, Hkv, D, causal), atol=0.02)


@pytest.mark.parametrize("M,N,Kd", [(2, 3072, 3072), (17, 3072, 8192), (64, 4096, 1024), (64, 8192, 512),
                                    (65, 3072, 3072), (128, 3072, 8192), (100, 8192, 512)])
def test_gemm_resid_rmsnorm_fused(M, N, Kd):
    torch.manual_seed(M + N)
    a, w = _rand(M, Kd), _rand(N, Kd, scale=Kd ** -0.5)
    x = _rand(M, N)
    g = _rand(N) + 1.0
    x_ref = x.clone()
    h = K.gemm_resid_norm(a, w, x, g, 1e-5, out=x)
    h_ref = R.gemm_resid_norm(a, w, x_ref, g, 1e-5, out=x_ref)
    _close(x, x_ref, atol=0.03)
    _close(h, h_ref, atol=0.05)


@pytest.mark.parametrize("tile,M", [(2, 64), (2, 40), (3, 17), (2, 130), (9, 128), (9, 77)])
@pytest.mark.parametrize("splits,Kd,N", [(1, 64, 392), (1, 448, 392), (2, 768, 392), (4, 3072, 392), (3, 576, 392),
                                         (2, 3072, 9216)])
def test_gemm_decode_tile(tile, M, splits, Kd, N):
    """Decode tiles with 4 k-tiles in flight (incl. nk < 4 and nk % 4 != 0) for every epilogue route
    (residual, SwiGLU, split-K partials + reduce, the fused reduce + RMSNorm) vs fp32."""
    torch.manual_seed(M + Kd + N)
    a, w, r = _rand(M, Kd), _rand(N, Kd, scale=Kd ** -0.5), _rand(M, N)
    g = _rand(N) + 1.0
    _close(K.gemm(a, w, epi=K.EPI_RESID, resid=r, tile=tile, splits=splits), R.gemm(a, w, epi=K.EPI_RESID, resid=r),
           atol=0.03)
    if N % 32 == 0:
        _close(K.gemm(a, w, epi=K.EPI_SWIGLU, tile=tile, splits=splits), R.gemm(a, w, epi=K.EPI_SWIGLU), atol=0.03)
    if (M <= 64 or (tile == 9 and M <= 128)) and N <= 8192:
        x, xr = r.clone(), r.clone()
        h = K.gemm_resid_norm(a, w, x, g, 1e-5, out=x, tile=tile, splits=splits)
        hr = R.gemm_resid_norm(a, w, xr, g, 1e-5, out=xr)
        _close(x, xr, atol=0.03)
        _close(h, hr, atol=0.05)


@pytest.mark.parametrize("M", [65, 128, 261, 1023])
def test_gemm_mid_m(M):
    """65..1023 rows (mid-size decode batches, short prefills) on the in-tree tiles (plain, residual
    in and out of place, gate/up + SwiGLU, and the explicit 128x128 tile) match the fp32 reference."""
    torch.manual_seed(M)
    N, F, Kd = 384, 256, 512
    a, w = _rand(M, Kd), _rand(N, Kd, scale=Kd ** -0.5)
    ref = a.float() @ w.float().t()
    _close(K.gemm(a, w), ref, atol=0.03)
    resid = _rand(M, N)
    _close(K.gemm(a, w, epi=K.EPI_RESID, resid=resid.clone(), out=None), ref + resid.float(), atol=0.05)
    x = resid.clone()
    K.gemm(a, w, epi=K.EPI_RESID, resid=x, out=x)  # in-place residual add
    _close(x, ref + resid.float(), atol=0.05)
    gate, up = _rand(F, Kd, scale=Kd ** -0.5), _rand(F, Kd, scale=Kd ** -0.5)
    got = K.gemm(a, R.interleave_gate_up(gate, up), epi=K.EPI_SWIGLU)
    _close(got, torch.nn.functional.silu(a.float() @ gate.float().t()) * (a.float() @ up.float().t()), atol=0.03)
    _close(K.gemm(a, w, tile=1), ref, atol=0.03)


@pytest.mark.parametrize("H,Hkv,D,P", [(32, 32, 96, 261), (8, 2, 128, 64), (4, 4, 64, 1), (4, 2, 96, 130),
                                       (32, 32, 96, 256), (4, 2, 96, 64)])
def test_flash_attn_shared_prefix(H, Hkv, D, P):
    """Suffix queries attend to P shared-prefix keys held in a KV-cache slot + their own keys (causal
    D = 96: the LDS-DMA pipelined kernel for whole 64-key prefixes, its register-staged form else)."""
    torch.manual_seed(H + D + P)
    lens = [1, 63, 64, 200, 7]
    T = sum(lens)
    qkv = _rand(T, (H + 2 * Hkv) * D)
    q, k, v = qkv[:, :H * D], qkv[:, H * D:(H + Hkv) * D], qkv[:, (H + Hkv) * D:]
    cu = torch.tensor([0] + list(np.cumsum(lens)), device=DEV, dtype=torch.int32)
    kc, vc = _rand(3, Hkv, 512, D), _rand(3, Hkv, 512, D)
    pre = (kc[1], vc[1], P)
    got = K.flash_attn_varlen(q, k, v, cu, max(lens), H, Hkv, D, True, prefix=pre)
    ref = R.flash_attn_varlen(q, k, v, cu, max(lens), H, Hkv, D, True, prefix=pre)
    _close(got, ref, atol=0.02)


@pytest.mark.parametrize("H,Hkv,P", [(32, 32, 0), (32, 32, 256), (8, 4, 64), (8, 2, 100)])
def test_flash_attn_kv_from_cache(H, Hkv, P):
    """The prefill as the model runs it for D = 96: the QKV epilogue writes k / v to the cache only
    (kv_out=False: the q columns and the caches are bit-identical to kv_out=True), and the attention
    reads each sequence's own keys from its cache slot at its first token's position — bit-identical
    to the attention over the k / v columns, with and without a shared prefix in another slot."""
    torch.manual_seed(H + P)
    D, Kd, S, L = 96, 256, 6, 1024
    lens = [300, 1, 64, 257, 90]
    T = sum(lens)
    N = (H + 2 * Hkv) * D
    a, w = _rand(T, Kd), _rand(N, Kd, scale=Kd ** -0.5)
    cu = torch.tensor([0] + list(np.cumsum(lens)), device=DEV, dtype=torch.int32)
    slot = torch.cat([torch.full((n,), b, dtype=torch.int32) for b, n in enumerate(lens)]).to(DEV)
    pos = torch.cat([torch.arange(P, P + n, dtype=torch.int32) for n in lens]).to(DEV)
    cs = R.rope_table(L, D, 10000.0, device=DEV)
    kc, vc = _rand(S, Hkv, L, D), _rand(S, Hkv, L, D)  # slot 5: the shared prefix's keys
    kc2, vc2 = kc.clone(), vc.clone()
    qkv = K.gemm_rope(a, w, pos, cs, H, Hkv, D, slot, kc, vc)
    qkv2 = K.gemm_rope(a, w, pos, cs, H, Hkv, D, slot, kc2, vc2, kv_out=False)
    assert torch.equal(qkv[:, :H * D], qkv2[:, :H * D]) and torch.equal(kc, kc2) and torch.equal(vc, vc2)
    pre = (kc[5], vc[5], P) if P else None
    q, k, v = qkv[:, :H * D], qkv[:, H * D:(H + Hkv) * D], qkv[:, (H + Hkv) * D:]
    ref = K.flash_attn_varlen(q, k, v, cu, max(lens), H, Hkv, D, True, prefix=pre)
    got = K.flash_attn_varlen(qkv2[:, :H * D], None, None, cu, max(lens), H, Hkv, D, True, prefix=pre,
                              kv_cache=(kc2, vc2, slot, pos))
    assert torch.equal(got, ref)
    _close(got, R.flash_attn_varlen(q, k, v, cu, max(lens), H, Hkv, D, True, prefix=pre), atol=0.02)


@pytest.mark.parametrize("H,Hkv,D", [(32, 32, 96), (32, 8, 128), (8, 1, 128), (12, 6, 64)])
def test_decode_attn_shared_prefix(H, Hkv, D):
    """Rows whose keys [0, P) live in a shared prefix slot (pre = (P, slot)) vs the fp32 reference."""
    torch.manual_seed(H + D)
    B, S = 5, 700
    kc, vc = _rand(7, Hkv, S, D), _rand(7, Hkv, S, D)
    lens = torch.tensor([64, 65, 300, 700, 129], device=DEV, dtype=torch.int32)
    slot = torch.tensor([6, 0, 3, 2, 1], device=DEV, dtype=torch.int32)
    pre = torch.tensor([[64, 5], [64, 5], [256, 5], [0, 0], [128, 4]], device=DEV, dtype=torch.int32)
    q = _rand(B, (H + 2 * Hkv) * D)
    got = K.decode_attn(q, kc, vc, lens, slot, H, Hkv, D, max_len=700, chunk=128, pre=pre)
    ref = R.decode_attn(q, kc, vc, lens, slot, H, Hkv, D, pre=pre)
    _close(got, ref, atol=0.02)


@pytest.mark.parametrize("fused", [False, True])
def test_decode_attn_split_merge(fused, monkeypatch):
    """In-kernel (last split merges, uncached partials) and separate-launch split merge vs reference."""
    monkeypatch.setattr(K, "_FUSED_COMBINE", fused)
    torch.manual_seed(3)
    H = Hkv = 32
    D, B, S = 96, 3, 1100
    kc, vc = _rand(4, Hkv, S, D), _rand(4, Hkv, S, D)
    lens = torch.tensor([1, 513, 1100], device=DEV, dtype=torch.int32)
    slot = torch.tensor([3, 0, 2], device=DEV, dtype=torch.int32)
    q = _rand(B, (H + 2 * Hkv) * D)
    ref = R.decode_attn(q, kc, vc, lens, slot, H, Hkv, D)
    for ch in (64, 512, 1152):
        _close(K.decode_attn(q, kc, vc, lens, slot, H, Hkv, D, max_len=S, chunk=ch), ref, atol=0.02)


@pytest.mark.parametrize("M", [2, 16, 17, 33, 64])
@pytest.mark.parametrize("N,Kd,epi", [(9216, 3072, 0), (3072, 3072, 4), (16384, 3072, 3), (3072, 8192, 4),
                                      (32064, 3072, 0), (512, 256, 1), (1024, 512, 3), (12320, 512, 3)])
def test_gemm_dk_matches_reference(M, N, Kd, epi):
    """gemm_dk (K split inside the workgroup, no split-K partials) == the fp32 reference for every
    epilogue and tile width (BN 16 / 32 / 64 from N), ragged M."""
    torch.manual_seed(M * 7 + N + Kd)
    a, w = _rand(M, Kd), _rand(N, Kd, scale=Kd ** -0.5)
    bias = _rand(N) if epi == 1 else None
    r = _rand(M, N) if epi == 4 else None
    got = K.gemm_dk(a, w, epi=epi, bias=bias, resid=r)
    _close(got, R.gemm(a, w, bias=bias, epi=epi, resid=r), atol=0.03)
    if K.dk_fusable(M, N, Kd, epi):  # the auto route of gemm() takes gemm_dk for 2..32 rows
        assert torch.equal(K.gemm(a, w, epi=epi, resid=r, bias=bias), got)


@pytest.mark.parametrize("M", [3, 16, 40, 64])
@pytest.mark.parametrize("H,F", [(3072, 8192), (4096, 14336)])
def test_gemm_dk_deferred_norm_chain(M, H, F):
    """Producer (EPI_RESID + per-part sums of squares) -> consumer (deferred RMSNorm of its A rows)
    == residual add, rmsnorm kernel, plain GEMM; the sums match the fp32 row sums."""
    torch.manual_seed(M + H)
    a, wo = _rand(M, H), _rand(H, H, scale=H ** -0.5)
    x = _rand(M, H)
    wgu = _rand(2 * F, H, scale=H ** -0.5)
    x_ref = x.clone()
    ssq = torch.zeros(512 * 64, dtype=torch.float32, device=DEV)
    parts = K.dk_parts(H, M)  # 33..64 rows: the split-K route's 512-column parts
    K.gemm_dk(a, wo, epi=K.EPI_RESID, resid=x, out=x, ssq_out=ssq)
    y = R.gemm(a, wo, epi=K.EPI_RESID, resid=x_ref)
    _close(x, y, atol=0.03)
    sums = ssq.view(-1, 64)[:parts, :M].sum(0)
    _close(sums, x.float().pow(2).sum(-1), atol=1e-2 * H, rtol=1e-3)
    g = K.gemm_dk(x, wgu, epi=K.EPI_SWIGLU, norm_in=(ssq, parts, 1e-5))
    h = K.rmsnorm(x, torch.ones(H, dtype=torch.bfloat16, device=DEV), 1e-5)
    _close(g, R.gemm(h, wgu, epi=K.EPI_SWIGLU), atol=0.03)
    # R.gemm_dk (the CPU model path) agrees with the kernel
    ssq_r = torch.zeros_like(ssq)
    x2 = x_ref.clone()
    R.gemm_dk(a, wo, epi=K.EPI_RESID, resid=x2, out=x2, ssq_out=ssq_r)
    _close(ssq_r.view(-1, 64)[:parts, :M], ssq.view(-1, 64)[:parts, :M], atol=0.5, rtol=2e-2)
    _close(R.gemm_dk(x, wgu, epi=K.EPI_SWIGLU, norm_in=(ssq, parts, 1e-5)), g, atol=0.03)
