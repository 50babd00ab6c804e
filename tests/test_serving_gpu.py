"""Serving-lane concurrency on the GPU: the continuous decode scheduler (graph replays on the GPU
thread), the fast embed lane (its own stream + kernel workspace) and the search plane (its own
thread, stream and workspace) running AT THE SAME TIME must produce exactly what each produces
alone. Regression test: the search plane once shared the GPU thread's split-K workspace, whose
pointer the decode graph had captured; concurrent top-k partials and GEMM partials corrupted each
other and a corrupted row index faulted the id gather."""
import concurrent.futures as cf
import threading

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from docagents_amd.engine.engine import Engine  # noqa: E402
from docagents_amd.ops import kernels as K  # noqa: E402
from docagents_amd.parallel.search_plane import SearchPlane  # noqa: E402


def test_decode_fast_embed_and_search_plane_co_run_exactly():
    dev = torch.device("cuda", 0)
    eng = Engine("bge-small", "tiny-dec", dev, max_batch=8, max_seq=1024, max_new_tokens=24, summary_max_new=8,
                 temperature=0.2)
    rng = np.random.default_rng(0)
    d = eng.dim
    X = rng.standard_normal((3000, d)).astype(np.float32)
    X /= np.linalg.norm(X, axis=1, keepdims=True)
    docs = [f"doc{i}" for i in range(300)]
    eng.index.add_bulk(docs, [10] * 300, np.arange(3000, dtype=np.int64) + 7000, torch.from_numpy(X))
    plane = SearchPlane(eng.index, 0, 1, device=dev).start()
    Q = rng.standard_normal((64, d)).astype(np.float32)
    Q /= np.linalg.norm(Q, axis=1, keepdims=True)
    # wide filters (the dense MFMA scan + bitmap path) and narrow ones (row ranges)
    flt = [[docs[j] for j in rng.choice(300, size=120 if i % 2 else 4, replace=False)] for i in range(64)]
    items = [(i, (f"question {i}?", [list(range(100 + i, 400 + i))], 0.9)) for i in range(12)]
    texts = [f"a short question number {i} about memory" for i in range(16)]

    def searches():
        return [plane.submit(Q[i:i + 8], 5, -1.0, flt[i:i + 8]).result(60) for i in range(0, 64, 8)]

    def answers():
        out, busy = eng.cb_tick(items, steps=4)
        res = dict((t, (a, c)) for t, a, c in out)
        while busy:
            o, busy = eng.cb_tick([], steps=16)
            res.update((t, (a, c)) for t, a, c in o)
        return [res[i] for i in range(12)]

    fast = torch.cuda.Stream(priority=-1)

    def embeds():
        with torch.cuda.stream(fast), K.workspace_role("fast"):
            return [eng.embed([t], False, out_dtype=torch.float32).cpu().numpy() for t in texts]

    # alone, one after the other
    s_ref, a_ref, e_ref = searches(), answers(), embeds()
    torch.cuda.synchronize()
    # together, three threads, three streams, three workspaces
    with cf.ThreadPoolExecutor(3) as ex:
        fa = ex.submit(answers)
        fs = ex.submit(lambda: [searches() for _ in range(3)])
        fe = ex.submit(lambda: [embeds() for _ in range(2)])
        a_got, s_got, e_got = fa.result(180), fs.result(180), fe.result(180)
    torch.cuda.synchronize()
    assert a_got == a_ref
    for rep in s_got:
        for (s0, k0), (s1, k1) in zip(s_ref, rep):
            assert np.array_equal(k0, k1) and np.allclose(s0, s1, atol=0, rtol=0)
    for rep in e_got:
        for v0, v1 in zip(e_ref, rep):
            assert np.array_equal(v0, v1)
    assert plane.healthy
    plane.stop()
    assert threading.active_count() >= 1


def test_release_decoder_returns_the_kv_cache_to_the_device():
    """bench.py's N > 1 blocks build TP decoders only after Engine.release_decoder: the KV cache
    (sized by parallel/hbm_plan.kv_bytes, the formula the plan uses) must really go back to the
    device, the weights stay (the TP blocks shard them) and embeds still work."""
    import torch

    from docagents_amd.engine.engine import Engine
    from docagents_amd.parallel.hbm_plan import kv_bytes
    eng = Engine("tiny-enc", "tiny-dec", "cuda:0", max_batch=8, max_seq=4096, max_new_tokens=4)
    eng.answer_many([("q?", [[5, 6, 7]], 0.5)], 4)  # a captured decode graph holds the cache too
    torch.cuda.synchronize()
    before = torch.cuda.memory_allocated()
    want = kv_bytes(eng.dec_cfg, 8 + 4, 4096)
    stats = eng.release_decoder()
    after = torch.cuda.memory_allocated()
    assert stats["decode_steps"] > 0 and eng.gen is None and eng.decoder.cache is None
    assert before - after >= want, (before, after, want)
    assert eng.decoder.w["layers"], "weights are kept"
    v = eng.embed(["still embeds"])
    assert v.shape == (1, eng.dim)
