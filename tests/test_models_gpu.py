"""Model-level numerics on the GPU: the HIP-kernel path vs the fp32-PyTorch reference path on the
same weights, plus HIP-graph decode vs eager decode."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from docagents_amd.engine.generator import Generator  # noqa: E402
from docagents_amd.models.bert import BertEncoder  # noqa: E402
from docagents_amd.models.configs import decoder_config, encoder_config  # noqa: E402
from docagents_amd.models.llama import LlamaDecoder, pack_prompts  # noqa: E402
from docagents_amd.ops import reference  # noqa: E402


def _to(w, dev):
    if isinstance(w, dict):
        return {k: _to(v, dev) for k, v in w.items()}
    if isinstance(w, list):
        return [_to(v, dev) for v in w]
    return w.to(dev)


def test_encoder_matches_reference():
    cfg = encoder_config("tiny-enc")
    enc = BertEncoder(cfg, "cuda", seed=3)
    ref = BertEncoder(cfg, "cuda", weights=enc.w)
    ref.ops = reference
    seqs = [list(range(5, 5 + n)) for n in (3, 70, 130, 1)]
    a = enc.encode_packed(seqs)
    b = ref.encode_packed(seqs)
    assert torch.allclose(a, b.to(a.device), atol=3e-2), (a - b).abs().max()
    cos = (a * b).sum(-1)
    assert cos.min() > 0.999


def test_decoder_prefill_matches_reference():
    cfg = decoder_config("tiny-dec")
    m = LlamaDecoder(cfg, "cuda", seed=1)
    m.alloc_cache(4, 512)
    r = LlamaDecoder(cfg, "cuda", weights=m.w)
    r.ops = reference
    r.alloc_cache(4, 512)
    prompts = [list(range(10, 10 + n)) for n in (5, 100, 33)]
    flat, pos, cu, lens = pack_prompts(prompts)
    slot_tok = np.repeat(np.arange(3, dtype=np.int32), lens)
    to = lambda x: torch.from_numpy(np.ascontiguousarray(x)).cuda()  # noqa: E731
    last = to((cu[1:] - 1).astype(np.int64))
    la = m.prefill(to(flat), to(pos), to(slot_tok), to(cu), int(lens.max()), last)
    lb = r.prefill(to(flat), to(pos), to(slot_tok), to(cu), int(lens.max()), last)
    assert (la.float() - lb.float()).abs().max() < 0.05
    assert torch.allclose(m.cache.buf.float(), r.cache.buf.float(), atol=0.05)


def test_generate_graph_equals_eager_greedy():
    cfg = decoder_config("tiny-dec")
    m = LlamaDecoder(cfg, "cuda", seed=2)
    m.alloc_cache(9, 512)
    g1 = Generator(m, max_batch=8, max_seq=512, temperature=0.0, use_graphs=True)
    prompts = [list(range(20, 20 + n)) for n in (7, 50, 3)]
    out1 = g1.generate(prompts, 12)
    m2 = LlamaDecoder(cfg, "cuda", weights=m.w)
    m2.alloc_cache(9, 512)
    g2 = Generator(m2, max_batch=8, max_seq=512, temperature=0.0, use_graphs=False)
    out2 = g2.generate(prompts, 12)
    for a, b in zip(out1, out2):
        assert a.tokens == b.tokens
        assert abs(a.mean_prob - b.mean_prob) < 1e-4
        assert len(a.tokens) == 12


def test_generate_matches_reference_greedy():
    cfg = decoder_config("tiny-dec")
    m = LlamaDecoder(cfg, "cuda", seed=4)
    m.alloc_cache(5, 256)
    g = Generator(m, max_batch=4, max_seq=256, temperature=0.0, use_graphs=True)
    r = LlamaDecoder(cfg, "cuda", weights=m.w)
    r.ops = reference
    r.alloc_cache(5, 256)
    gr = Generator(r, max_batch=4, max_seq=256, temperature=0.0, use_graphs=False)
    gr.is_cuda = False
    prompts = [list(range(40, 60)), list(range(3, 9))]
    a, b = g.generate(prompts, 6), gr.generate(prompts, 6)
    agree = sum(x == y for p, q in zip(a, b) for x, y in zip(p.tokens, q.tokens))
    assert agree >= 10  # bf16 vs fp32 may flip a near-tie late in the sequence


def test_generate_shared_prompt_head_matches_unshared():
    """Shared-head prefill (head once, suffixes vs cached head keys) and decode (every row reads the
    head's keys from the one slot holding them) generate what the plain per-prompt path generates
    (bf16: allow rare near-tie flips)."""
    m = LlamaDecoder(decoder_config("tiny-dec"), "cuda", seed=6)
    m.alloc_cache(9, 1024)
    g = Generator(m, max_batch=8, max_seq=1024, temperature=0.0, use_graphs=True)
    rng = np.random.default_rng(11)
    head = [int(t) for t in rng.integers(5, 3000, size=261)]
    prompts = [head + [int(t) for t in rng.integers(5, 3000, size=n)] for n in (1, 300, 45, 128, 9)]
    g.share_prefix = False
    want = g.generate(prompts, 12)
    g.share_prefix = True
    got = g.generate(prompts, 12)
    assert g.stats["shared_prefix_tokens"] == 256 * 4
    agree = np.mean([np.mean([x == y for x, y in zip(a.tokens, b.tokens)]) for a, b in zip(got, want)])
    assert agree >= 0.75, agree
    assert max(abs(a.mean_prob - b.mean_prob) for a, b in zip(got, want)) < 0.02


def test_continuous_scheduler_prompt_head_cache_graphs():
    """Graph-replayed continuous batching with a cached prompt head: same tokens as per-prompt runs."""
    from docagents_amd.engine.generator import ContinuousScheduler
    m = LlamaDecoder(decoder_config("tiny-dec"), "cuda", seed=8)
    m.alloc_cache(8, 1024)
    g = Generator(m, max_batch=4, max_seq=1024, temperature=0.0, use_graphs=True)
    rng = np.random.default_rng(12)
    head = [int(t) for t in rng.integers(5, 3000, size=300)]
    prompts = [head + [int(t) for t in rng.integers(5, 3000, size=n)] for n in (5, 64, 200, 17, 90)]
    g.share_prefix = False
    want = [g.generate([p], 8)[0] for p in prompts]
    g.share_prefix = True
    sched = ContinuousScheduler(g, B=4, max_new_cap=8, chunk_steps=4)
    res = sched.run_all(prompts, 8)
    assert sched.stats["heads_built"] == 1 and sched.stats["head_hits"] == 5
    agree = np.mean([np.mean([x == y for x, y in zip(a.tokens, b.tokens)]) for a, b in zip(res, want)])
    assert agree >= 0.75, agree


def _near_argmax_under_reference(r, prompt, gen, margin=0.1):
    """Teacher-forced check of a generated sequence against the fp32 reference model: every token the
    HIP path chose is within ``margin`` (log-prob) of the reference's best token given the same
    history. A wrong kernel picks essentially random tokens (several nats below the best); a bf16
    near-tie flip stays inside the margin."""
    worst = 0.0
    for t, tok in enumerate(gen):
        seq = prompt + gen[:t]
        to = lambda x: torch.from_numpy(np.ascontiguousarray(x)).cuda()  # noqa: E731
        flat = np.asarray(seq, dtype=np.int32)
        lg = r.prefill(to(flat), to(np.arange(len(seq), dtype=np.int32)), to(np.zeros(len(seq), dtype=np.int32)),
                       to(np.array([0, len(seq)], dtype=np.int32)), len(seq), to(np.array([len(seq) - 1])))
        lp = torch.log_softmax(lg[0].float(), -1)
        worst = max(worst, float(lp.max() - lp[tok]))
    assert worst <= margin, worst
    return worst


def _width_model(name, layers=2, seed=5, slots=6, max_seq=1024):
    import dataclasses
    cfg = dataclasses.replace(decoder_config(name), layers=layers)
    m = LlamaDecoder(cfg, "cuda", seed=seed)
    m.alloc_cache(slots, max_seq)
    r = LlamaDecoder(cfg, "cuda", weights=m.w)
    r.ops = reference
    r.alloc_cache(2, max_seq)
    return m, r


def test_phi3_width_prefill_and_decode_vs_reference():
    """Phi-3-mini at full width (hidden 3072, 32 MHA heads of D = 96, FFN 8192), 2 layers: the
    production kernels — phase-split QKV GEMM with the RoPE + KV-cache epilogue, gemm8p SwiGLU / residual
    GEMMs, causal flash attention, HIP-graph decode with fused-RoPE decode attention and the
    gemm_resid_norm layer tail (batch 3), and the fused-RMSNorm GEMV path (batch 1) — vs fp32."""
    m, r = _width_model("phi3-mini")
    prompts = [[int(t) for t in np.random.default_rng(i).integers(5, 32000, size=n)] for i, n in enumerate((300, 129, 64))]
    flat, pos, cu, lens = pack_prompts(prompts)
    to = lambda x: torch.from_numpy(np.ascontiguousarray(x)).cuda()  # noqa: E731
    slot_tok = np.repeat(np.arange(3, dtype=np.int32), lens)
    last = to((cu[1:] - 1).astype(np.int64))
    la = m.prefill(to(flat), to(pos), to(slot_tok), to(cu), int(lens.max()), last)
    rr = LlamaDecoder(m.cfg, "cuda", weights=m.w)
    rr.ops = reference
    rr.alloc_cache(6, 1024)
    lb = rr.prefill(to(flat), to(pos), to(slot_tok), to(cu), int(lens.max()), last)
    assert (la.float() - lb.float()).abs().max() < 0.08, (la.float() - lb.float()).abs().max()
    assert torch.allclose(m.cache.buf[:, :, :3].float(), rr.cache.buf[:, :, :3].float(), atol=0.06)
    g = Generator(m, max_batch=4, max_seq=1024, temperature=0.0, use_graphs=True)
    outs = g.generate(prompts, 8)
    for p, o in zip(prompts, outs):
        _near_argmax_under_reference(r, p, o.tokens)
    one = g.generate([prompts[2]], 8)[0]  # batch 1: fused-RMSNorm GEMV decode
    _near_argmax_under_reference(r, prompts[2], one.tokens)


def test_bge_base_width_encoder_vs_reference():
    """BGE-base at full width (hidden 768, 12 heads of D = 64, FFN 3072), 2 layers: LayerNorm,
    bias / GELU GEMM epilogues, bidirectional flash attention, CLS pooling + L2 norm vs fp32."""
    import dataclasses
    cfg = dataclasses.replace(encoder_config("bge-base"), layers=2)
    enc = BertEncoder(cfg, "cuda", seed=3)
    ref = BertEncoder(cfg, "cuda", weights=enc.w)
    ref.ops = reference
    seqs = [[int(t) for t in np.random.default_rng(n).integers(1000, 30000, size=n)] for n in (512, 300, 17, 1, 129)]
    a = enc.encode_packed(seqs)
    b = ref.encode_packed(seqs).to(a.device)
    cos = (a.float() * b.float()).sum(-1)
    assert cos.min() > 0.999, cos
    assert torch.allclose(a.float(), b.float(), atol=3e-2)


@pytest.mark.parametrize("arch,dtype", [("tiny-enc", "bf16"), ("bge-base", "bf16"), ("tiny-enc", "fp16"),
                                        ("tiny-enc", "fp8")])
def test_encoder_one_sequence_graphs_match_eager(arch, dtype):
    """encode_one (length-bucket HIP graphs, padded rows past the real length) == the eager packed
    path (and, bf16, the fp32 reference) across bucket edges and repeated replays; the capture works
    for every encoder dtype (the engine captures at startup)."""
    import dataclasses
    cfg = encoder_config(arch)
    if arch == "bge-base":
        cfg = dataclasses.replace(cfg, layers=2)
    enc = BertEncoder(cfg, "cuda", seed=5, dtype=dtype)
    enc.prepare_graphs()
    assert set(enc._g) == set(BertEncoder.GRAPH_BUCKETS)
    ref = None
    if dtype == "bf16":
        ref = BertEncoder(cfg, "cuda", weights=enc.w)
        ref.ops = reference
    for n in (1, 2, 15, 16, 17, 31, 33, 64, 100, 128, 129, 20, 1):
        seq = [int(t) for t in np.random.default_rng(n).integers(5, cfg.vocab - 1, size=n)]
        g = enc.encode_one(seq)
        e = enc.encode_packed([seq])
        assert g.shape == e.shape == (1, cfg.hidden)
        assert float((g.float() * e.float()).sum()) > 0.999, n
        if ref is not None:
            r = ref.encode_packed([seq]).to(g.device)
            assert torch.allclose(g.float(), r.float(), atol=3e-2), n


@pytest.mark.parametrize("arch,dtype", [("tiny-enc", "bf16"), ("bge-base", "bf16"), ("tiny-enc", "fp16"),
                                        ("tiny-enc", "fp8")])
def test_encoder_batch_graphs_match_eager(arch, dtype):
    """encode_batch (the fast lane's micro-batches through captured (sequences, tokens) bucket graphs:
    sequences packed, padding rows, zero-length padded sequences) == the eager packed path row by
    row, at every bucket edge; batches that fit no bucket return None (the caller goes eager)."""
    import dataclasses
    cfg = encoder_config(arch)
    if arch == "bge-base":
        cfg = dataclasses.replace(cfg, layers=2)
    enc = BertEncoder(cfg, "cuda", seed=7, dtype=dtype)
    enc.prepare_graphs()
    assert set(enc._gb) == {nb for nb, _ in BertEncoder.BATCH_BUCKETS}
    rng = np.random.default_rng(3)
    for n, lo, hi in [(2, 1, 30), (3, 5, 40), (4, 20, 31), (7, 3, 36), (16, 10, 31), (17, 2, 30), (33, 1, 31),
                      (64, 20, 31), (5, 100, 128)]:
        seqs = [[int(t) for t in rng.integers(5, cfg.vocab - 1, size=int(m))] for m in rng.integers(lo, hi + 1, size=n)]
        got = enc.encode_batch(seqs)
        if sum(map(len, seqs)) >= dict(BertEncoder.BATCH_BUCKETS)[64]:
            assert got is None
            continue
        assert got is not None and got.shape == (n, cfg.hidden), (n, lo, hi)
        want = enc.encode_packed(seqs)
        cos = (got.float() * want.float()).sum(-1)
        assert float(cos.min()) > 0.999, (n, lo, hi, cos.min())
    assert enc.encode_batch([[5] * 129, [6] * 3]) is None  # longer than the captured max_seqlen
    assert enc.encode_batch([[5] * 40] * 65) is None       # more sequences than the largest bucket


def test_encoder_one_sequence_graphs_two_streams_concurrent():
    """Two threads on two streams (the engine's fast embed lane and its GPU thread) call encode_one at
    once; the captured graphs share their static ids / cu / out buffers, so without device-side
    ordering one caller's input copy lands during the other's replay. Each thread's
    stream is first held busy (ops.spin) so the two streams' graph uses overlap on the device. Every
    result must equal the eager path for its own sequence."""
    import dataclasses
    import threading

    from docagents_amd.ops import kernels
    cfg = dataclasses.replace(encoder_config("bge-base"), layers=2)
    enc = BertEncoder(cfg, "cuda", seed=6)
    enc.prepare_graphs()
    rng = np.random.default_rng(11)
    seqs = [[int(t) for t in rng.integers(5, cfg.vocab - 1, size=int(n))] for n in rng.integers(3, 120, size=64)]
    want = [enc.encode_packed([s]).float() for s in seqs]
    torch.cuda.synchronize()
    got = [None] * len(seqs)
    lock = threading.Lock()  # the engine's enc_lock: host-side enqueue order only

    def worker(which):
        st = torch.cuda.Stream()
        with torch.cuda.stream(st):
            for i in range(which, len(seqs), 2):
                with lock:
                    kernels.spin(200 if i % 4 < 2 else 0)
                    got[i] = enc.encode_one(seqs[i])
        st.synchronize()
    ts = [threading.Thread(target=worker, args=(w,)) for w in (0, 1)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    torch.cuda.synchronize()
    bad = [i for i in range(len(seqs)) if float((got[i].float() * want[i]).sum()) < 0.999]
    assert not bad, bad


def test_generate_batch_above_64_graph_equals_eager():
    """Decode batches above 64 rows (mid-M weight-streaming tiles with split-K inside the captured
    graph): graph replay == eager, token for token, and near-argmax under the fp32 reference."""
    cfg = decoder_config("tiny-dec")
    m = LlamaDecoder(cfg, "cuda", seed=9)
    m.alloc_cache(130, 256)
    rng = np.random.default_rng(3)
    prompts = [[int(t) for t in rng.integers(5, 3000, size=int(n))] for n in rng.integers(3, 60, size=100)]
    g1 = Generator(m, max_batch=128, max_seq=256, temperature=0.0, use_graphs=True, share_prefix=False)
    out1 = g1.generate(prompts, 6)
    m2 = LlamaDecoder(cfg, "cuda", weights=m.w)
    m2.alloc_cache(130, 256)
    g2 = Generator(m2, max_batch=128, max_seq=256, temperature=0.0, use_graphs=False, share_prefix=False)
    out2 = g2.generate(prompts, 6)
    assert [o.tokens for o in out1] == [o.tokens for o in out2]
    r = LlamaDecoder(cfg, "cuda", weights=m.w)
    r.ops = reference
    r.alloc_cache(2, 256)
    for i in (0, 57, 99):
        _near_argmax_under_reference(r, prompts[i], out1[i].tokens)


def test_batch1_decode_folded_gains_matches_unfolded():
    """Batch-1 decode fuses RMSNorm into the QKV / gate-up / lm-head GEMVs. With the checkpoint's
    gains folded into those weights the GEMVs run gain-free (rms=(None, eps)); an unfolded model
    streams the gains. Both must generate the same greedy tokens."""
    import copy
    from docagents_amd.models.llama import random_weights

    class Unfolded(LlamaDecoder):
        def _fold_norm_gains(self):
            pass

    import dataclasses
    # hidden 512: the GEMV path needs K % 512 == 0 (tiny-dec's 256 would route to the tile GEMM)
    cfg = dataclasses.replace(decoder_config("tiny-dec"), name="tiny-dec-512", hidden=512, heads=8,
                              kv_heads=4, ffn=1024)
    w = random_weights(cfg, "cuda", seed=12)
    g = torch.Generator(device="cuda").manual_seed(5)
    for L in w["layers"]:
        for k in ("ln_attn", "ln_mlp"):
            L[k] = (0.5 + torch.rand(L[k].shape, generator=g, device="cuda")).to(torch.bfloat16)
    w["norm"] = (0.5 + torch.rand(w["norm"].shape, generator=g, device="cuda")).to(torch.bfloat16)
    m, u = LlamaDecoder(cfg, "cuda", weights=copy.deepcopy(w)), Unfolded(cfg, "cuda", weights=copy.deepcopy(w))
    assert m.unit_gains and not u.unit_gains
    assert m.ops.gemv_fusable(1, m.w["layers"][0]["wqkv"].shape[0], cfg.hidden)
    outs = []
    for mm in (m, u):
        mm.alloc_cache(3, 256)
        outs.append(Generator(mm, max_batch=2, max_seq=256, temperature=0.0, use_graphs=True)
                    .generate([list(range(50, 83))], 10)[0])
    a, b = outs
    assert sum(x == y for x, y in zip(a.tokens, b.tokens)) >= 8, (a.tokens, b.tokens)
    assert abs(a.mean_prob - b.mean_prob) < 0.05 * max(a.mean_prob, 1e-6) + 1e-4
