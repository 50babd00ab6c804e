"""Flash prefill dispatch order (attention.hip fa_block): grid order with causal longest-first
(da_set_flash_rev(1)) and the XCD-grouped (sequence, kv head) pairs (rev 3, the default) compute
the same bits — the order only moves where and when a block runs — for MHA / GQA, causal /
bidirectional, packed variable-length batches, a shared prompt head and a pair count that is not
a multiple of 8 (grouping falls back to grid order); each against the fp32 oracle too."""
import pytest
import torch

pytestmark = pytest.mark.gpu

from docagents_amd.ops import kernels as K  # noqa: E402
from docagents_amd.ops import reference as R  # noqa: E402

CASES = [  # name, lengths, H, Hkv, D, causal
    ("mha96_causal", [700] * 8, 32, 32, 96, True),
    ("gqa128_causal", [1000, 1000, 1000, 1000], 32, 8, 128, True),
    ("mha96_varlen", [1500, 37, 640, 900, 1, 1280, 333, 2047], 32, 32, 96, True),
    ("bert64", [512] * 8, 12, 12, 64, False),
    ("pairs_not_mult8", [300] * 3, 12, 12, 64, True),  # 36 pairs: grid order
]


@pytest.mark.parametrize("name,lens,H,Hkv,D,causal", CASES, ids=[c[0] for c in CASES])
def test_flash_dispatch_order_bit_identical(name, lens, H, Hkv, D, causal):
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(len(name))
    T = sum(lens)
    qkv = torch.randn(T, (H + 2 * Hkv) * D, device=dev, generator=g).to(torch.bfloat16)
    q, k, v = qkv[:, :H * D], qkv[:, H * D:(H + Hkv) * D], qkv[:, (H + Hkv) * D:]
    cu = torch.tensor([0] + list(torch.tensor(lens).cumsum(0)), dtype=torch.int32, device=dev)
    outs = {}
    try:
        for rev in (1, 3):
            K.lib().da_set_flash_rev(rev)
            outs[rev] = K.flash_attn_varlen(q, k, v, cu, max(lens), H, Hkv, D, causal=causal)
        torch.cuda.synchronize()
    finally:
        K.lib().da_set_flash_rev(3)
    assert torch.equal(outs[1], outs[3])
    ref = R.flash_attn_varlen(q, k, v, cu, max(lens), H, Hkv, D, causal=causal)
    assert (outs[3].float() - ref.float()).abs().max() < 0.03


def test_flash_dispatch_order_shared_head():
    """Keys [0, P) of every sequence from a shared prompt head in the KV cache (the QA prefill's
    kept system prompt): both dispatch orders, the same bits."""
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(3)
    H = Hkv = 32
    D, P, S = 96, 128, 2048
    lens = [600, 700, 650, 500, 720, 610, 590, 640]
    T = sum(lens)
    qkv = torch.randn(T, 3 * H * D, device=dev, generator=g).to(torch.bfloat16)
    q, k, v = qkv[:, :H * D], qkv[:, H * D:2 * H * D], qkv[:, 2 * H * D:]
    kc = torch.randn(Hkv, S, D, device=dev, generator=g).to(torch.bfloat16)
    vc = torch.randn(Hkv, S, D, device=dev, generator=g).to(torch.bfloat16)
    cu = torch.tensor([0] + list(torch.tensor(lens).cumsum(0)), dtype=torch.int32, device=dev)
    outs = {}
    try:
        for rev in (1, 3):
            K.lib().da_set_flash_rev(rev)
            outs[rev] = K.flash_attn_varlen(q, k, v, cu, max(lens), H, Hkv, D, causal=True, prefix=(kc, vc, P))
        torch.cuda.synchronize()
    finally:
        K.lib().da_set_flash_rev(3)
    assert torch.equal(outs[1], outs[3])
