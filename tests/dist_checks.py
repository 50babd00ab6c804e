"""Multi-process correctness checks for the distributed paths (test harness: run with gloo on CPU,
or with GPU ranks through gpurun). Each ``check_*`` is a ``torch.multiprocessing.spawn`` target;
rank 0 writes a JSON verdict to ``out_path``. Imported by the tests as ``dist_checks`` (tests/ is on
sys.path under pytest, and spawned children inherit it).

  check_tp_decoder      TP=world LlamaDecoder (column/row-parallel + all-reduce, vocab-parallel
                        lm_head + all-gather) == the unsharded decoder (prefill logits, greedy tokens)
  check_sharded_index   W-way sharded flat index (C2 all-gather queries, C1 all-gather top-k, merge)
                        == exact single-index search over all rows, with doc filters and threshold
  check_replicas        independent replicas (DP or TP x DP) + the search plane: a slow replica
                        blocks nobody, owner-routed ingest, exact sharded search, load balancing
  check_ivf_kmeans      IVFFlat with cross-shard k-means statistics all-reduce (C6)
  check_xgmi_allreduce  IPC peer-buffer all-reduce kernel == fp32 rank-order sum (GPU ranks)
  check_tp_decoder_gpu  TP=world decoder on GPU ranks (xGMI all-reduce in every layer) vs unsharded
"""
from __future__ import annotations

import json
import os
import socket

import numpy as np
import torch
import torch.distributed as dist


def _init(rank, world, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    # world processes share the machine's cores: no intra-op thread oversubscription
    torch.set_num_threads(max(1, (os.cpu_count() or 1) // world))
    dist.init_process_group("gloo", rank=rank, world_size=world)


def _done(rank, out_path, verdict):
    if rank == 0:
        with open(out_path, "w") as f:
            json.dump(verdict, f)
    dist.barrier()
    dist.destroy_process_group()


def check_tp_decoder(rank, world, port, out_path, arch: str = "tiny-dec", wrong_order: bool = False):
    """TP=world decoder vs the unsharded one on the same weights, per decision
    (docagents_amd/parallel/tp_verify.py: teacher-forced logit bound d, every decision with a top-1 /
    top-2 gap above 2 d agreeing, identical free-running tokens up to each prompt's first undecidable
    step). ``wrong_order`` runs the negative control (neighbour's shard)."""
    _init(rank, world, port)
    from docagents_amd.parallel.tp_verify import decision_verdict
    _done(rank, out_path, decision_verdict(rank, world, None, "cpu", arch=arch, wrong_order=wrong_order))


def check_tp8_decoder(rank, world, port, out_path):
    """TP=world with one KV head per rank (Llama-3-70B's TP=8 layout, tiny-dec-tp8)."""
    check_tp_decoder(rank, world, port, out_path, arch="tiny-dec-tp8")


def check_tp_decoder_wrong_order(rank, world, port, out_path):
    """Negative control of check_tp_decoder: shards loaded in the wrong rank order."""
    check_tp_decoder(rank, world, port, out_path, wrong_order=True)


def check_distributed_sampling(rank, world, port, out_path):
    """C4: sampling over a vocab-parallel LM head (each rank: its [B, V/t] slice -> 8-float row
    summaries -> one all-gather -> finalize) == the sampler on the full rows: same tokens, same
    logprobs (to fp32 rounding of the log-sum-exp regrouping), same bookkeeping (pos / hist / conf /
    active), greedy and at T = 0.2 / 1.0, on every rank."""
    _init(rank, world, port)
    from docagents_amd.models.llama import TPContext, tp_sample
    from docagents_amd.ops import reference as R
    B, V = 6, 32064 // 8 * 8
    g = torch.Generator().manual_seed(11)
    logits = (torch.randn(B, V, generator=g) * 3).bfloat16()
    logits[0, 5] = logits[0, V - 3] = 40.0  # an exact tie across ranks: the lower index must win
    tp = TPContext(rank, world, None)
    Vl = V // world
    ok, worst = True, 0.0
    for T in (0.0, 0.2, 1.0):
        def state():
            return dict(out_tok=torch.zeros(B, dtype=torch.int32), out_lp=torch.zeros(B),
                        conf=torch.zeros(B, 2), active=torch.tensor([1, 1, 1, 0, 1, 1], dtype=torch.int32),
                        pos=torch.arange(B, dtype=torch.int32) + 100, lens=torch.arange(B, dtype=torch.int32) + 101,
                        hist=torch.full((B, 4), -1, dtype=torch.int32), start=torch.full((B,), 99, dtype=torch.int32))
        a, b = state(), state()
        R.sample(logits, T, 7, 0, ctr=a["pos"], eos=(3,), **a)
        tp_sample(R, tp, logits[:, rank * Vl:(rank + 1) * Vl].contiguous(), T, 7, 0, ctr=b["pos"], eos=(3,), **b)
        for k in a:
            if k in ("out_lp", "conf"):
                err = float((a[k] - b[k]).abs().max())
                worst = max(worst, err)
                ok &= err < 1e-4
            else:
                ok &= bool(torch.equal(a[k], b[k]))
        ok &= int(a["out_tok"][0]) == 5 if T == 0.0 else True
    oks = [None] * world
    dist.all_gather_object(oks, (ok, worst))
    _done(rank, out_path, {"ok": all(o for o, _ in oks), "max_lp_err": max(w for _, w in oks)})


def check_sharded_index(rank, world, port, out_path):
    _init(rank, world, port)
    from docagents_amd.index.flat import FlatIndex
    from docagents_amd.parallel.sharded_index import ShardedIndex
    d, per, B, k = 64, 120, 5, 7
    rng = np.random.default_rng(0)  # identical global data on every rank
    X = rng.standard_normal((world * per, d)).astype(np.float32)
    X /= np.linalg.norm(X, axis=1, keepdims=True)
    docs = [f"doc{i // 10}" for i in range(world * per)]
    local = FlatIndex(d, "cpu")
    for r0 in range(rank * per, (rank + 1) * per, 10):
        local.add(docs[r0], np.arange(r0, r0 + 10), torch.from_numpy(X[r0:r0 + 10]))
    sh = ShardedIndex(local, rank, world)
    Q = rng.standard_normal((world * B, d)).astype(np.float32)
    Q /= np.linalg.norm(Q, axis=1, keepdims=True)
    filters = [[f"doc{j}" for j in rng.choice(world * per // 10, size=4, replace=False)] for _ in range(world * B)]
    filters[0] = [docs[-1], docs[0]]
    s, ids = sh.search(torch.from_numpy(Q[rank * B:(rank + 1) * B]), k, 0.0, filters)
    # exact reference over all rows (bf16-rounded operands, like the index); ids must match except
    # where two candidates tie within bf16 rounding
    Xb = torch.from_numpy(X).bfloat16().float().numpy()
    Qb = torch.from_numpy(Q).bfloat16().float().numpy()
    ok = True
    s = s.numpy()
    for b in range(B):
        qi = rank * B + b
        allowed = np.array([docs[i] in filters[qi] for i in range(len(docs))])
        sc = Xb @ Qb[qi]
        m = allowed & (sc >= 0.0)
        idx = np.where(m)[0]
        order = idx[np.lexsort((idx, -sc[idx]))][:k]
        got = [int(i) for i in ids[b].tolist() if i >= 0]
        if len(got) != len(order) or not np.allclose(np.sort(s[b][:len(got)]), np.sort(sc[order]), atol=2e-3):
            ok = False
        if any(not allowed[i] for i in got):
            ok = False
        if sum(1 for x, y in zip(got, order.tolist()) if x != y) > 1:
            ok = False
    oks = [None] * world
    dist.all_gather_object(oks, ok)
    _done(rank, out_path, {"exact": all(oks)})


def check_replicas(rank, world, port, out_path, tp: int = 1):
    """Independent engine replicas (engine/server.py EngineGroup) + the cross-rank search plane,
    the whole serving stack per rank as engine_main builds it: world / tp replicas, each leader an
    RPC endpoint on base + replica, TP followers stepping with their leader, every rank one index
    shard. Replica 1's decode ticks are slowed to 3 s each (fault hook); while one of its answers
    is in flight, the other replicas must serve answers, embeds, searches (which need every rank's
    shard, replica 1's included) and fused embed+search well inside that time, and ingest routed
    by document owner must land on the owner's shard (followers included). Rank 0 drives through
    ``EngineCluster`` (topology discovery, least-loaded balancing, owner routing)."""
    import asyncio
    import time as _t
    _init(rank, world, port)
    from docagents_amd.engine.engine import Engine
    from docagents_amd.engine.rpc import EngineCluster
    from docagents_amd.engine.server import EngineGroup, EngineServer, owner_of
    from docagents_amd.models.llama import TPContext
    from docagents_amd.utils import faults
    from docagents_amd.utils.log import discard
    from docagents_amd.parallel.search_plane import SearchPlane
    replicas, replica = world // tp, rank // tp
    rep_ctrl = rep_data = None
    for r in range(replicas):
        ranks = list(range(r * tp, (r + 1) * tp))
        c = dist.new_group(ranks, backend="gloo") if tp > 1 else None
        d = dist.new_group(ranks, backend="gloo") if tp > 1 else None
        if r == replica:
            rep_ctrl, rep_data = c, d
    plane_ctrl = dist.new_group(backend="gloo")
    tpc = TPContext(rank % tp, tp, rep_data) if tp > 1 else None
    eng = Engine("tiny-enc", "tiny-dec-tp8" if tp > 1 else "tiny-dec", "cpu", tp=tpc, max_batch=4, max_seq=512,
                 max_new_tokens=4, summary_max_new=4, use_graphs=False)
    if replica == 1:
        faults.configure_delay({"engine.tick": float(os.environ.get("DA_TEST_SLOW_TICK", "3.0"))})
    plane = SearchPlane.start_world(eng.index, rank, world, plane_ctrl)
    grp = EngineGroup(eng, rank, world, rep_ctrl, rep_data, tp_size=tp, plane=plane)
    # replica endpoints: free ports picked by rank 0 (neighbours of the rendezvous port may already
    # be taken by the process group's own connections)
    ports = [0] * replicas
    if rank == 0:
        socks = [socket.socket() for _ in range(replicas)]
        for sk in socks:
            sk.bind(("127.0.0.1", 0))
        ports = [sk.getsockname()[1] for sk in socks]
        for sk in socks:
            sk.close()
    box = [ports]
    dist.broadcast_object_list(box, src=0)
    urls = [f"tcp://127.0.0.1:{p}" for p in box[0]]
    done_flag = out_path + ".done"
    if not grp.is_leader:
        grp.follower_loop()
        plane.stop()
        dist.barrier()
        dist.destroy_process_group()
        return

    async def serve():
        srv = EngineServer(grp, discard(), continuous=True, cb_window_s=0.0, urls=urls, liveness_s=0)
        await srv.start(urls[replica])
        if rank == 0:
            verdict = await drive()
            with open(out_path, "w") as f:
                json.dump(verdict, f)
            open(done_flag, "w").close()
        else:
            while not os.path.exists(done_flag):
                await asyncio.sleep(0.05)
        srv.server.close()
        if tp > 1:
            grp._bcast(("shutdown", {}))

    async def drive():
        v = {}
        cl = await EngineCluster(urls[0]).connect(retries=200, delay=0.05)
        v["replicas"] = cl.replicas
        # ingest routed by owner (followers own shards too under TP)
        docs, per = [], {}
        i = 0
        while len(docs) < 4 * world or min(per.get(r, 0) for r in range(world)) < 2:  # every shard owns docs
            d = f"doc-{i}"
            i += 1
            o = owner_of(d, world)
            if per.get(o, 0) < 4:
                docs.append(d)
                per[o] = per.get(o, 0) + 1
        texts = {d: [f"chunk {j} of {d} about subject {i * 3 + j}" for j in range(3)] for i, d in enumerate(docs)}
        counts = await asyncio.gather(*[cl.call("embed_index", doc_id=d, keys=np.arange(3, dtype=np.int64) + 10 * i,
                                                texts=texts[d]) for i, d in enumerate(docs)])
        have = await cl.call("index_docs")
        v["ingest_ok"] = [int(r["rows"]) for r in counts] == [3] * len(docs) and all(have.get(d) == 3 for d in docs)
        v["owners"] = sorted({owner_of(d, world) for d in docs})
        # misrouted index mutation is rejected
        wrong = next(d for d in docs if owner_of(d, world) // tp != 0)
        try:
            await cl.clients[0].call("index_add", doc_id=wrong, keys=np.array([1]),
                                     vecs=np.ones((1, eng.dim), dtype=np.float32))
            v["misroute_rejected"] = False
        except Exception as e:  # noqa: BLE001
            v["misroute_rejected"] = "route index calls by owner" in str(e)
        # exact reference for searches: every chunk's vector (the fast-lane embed == the ingest embed)
        allt = [t for d in docs for t in texts[d]]
        allv = (await cl.clients[2 % cl.replicas].call("embed", texts=allt, preprocess=True))["vecs"]
        keys = [10 * i + j for i, _ in enumerate(docs) for j in range(3)]
        # slow replica 1: an answer that takes >= 3 s per tick
        slow = asyncio.ensure_future(cl.clients[1].call("answer", items=[{"question": "slow?", "context": "c",
                                                                             "quality": 1.0}]))
        await asyncio.sleep(0.3)
        t0 = _t.perf_counter()
        q = allv[[1, 7]].copy()
        flt = [[docs[0], docs[2]], docs[:]]
        others = [r for r in range(cl.replicas) if r != 1]
        jobs = [cl.clients[others[0]].call("search", vecs=q, filters=flt, k=4, min_sim=-1.0),
                cl.clients[others[-1]].call("embed_search", texts=[allt[7]], filters=[docs], k=3, min_sim=-1.0),
                cl.clients[others[-1]].call("embed", texts=["a question"], preprocess=True)]
        jobs += [cl.clients[r].call("answer", items=[{"question": f"q{r}?", "context": "ctx", "quality": 0.5}])
                 for r in others]
        async def timed(j):
            r_ = await j
            return r_, _t.perf_counter() - t0
        out = await asyncio.gather(*[timed(j) for j in jobs])
        res = [r_ for r_, _ in out]
        v["job_s"] = [round(x, 3) for _, x in out]
        v["others_s"] = _t.perf_counter() - t0
        v["slow_pending"] = not slow.done()
        def matches(qv, allowed_docs, k, s_row, k_row):
            """Exact brute-force top-k over every chunk (the random-init encoder maps all texts to
            nearby directions, so ids may swap only where scores tie within bf16 rounding)."""
            allowed = np.array([d in allowed_docs for d in docs for _ in range(3)])
            sc = allv @ qv
            idx = np.where(allowed)[0]
            order = idx[np.lexsort((idx, -sc[idx]))][:k]
            got = [int(x) for x in k_row if x >= 0]
            if len(got) != len(order) or not np.allclose(np.sort(s_row[:len(got)]), np.sort(sc[order]), atol=1e-2):
                return False
            pos = {kk: j for j, kk in enumerate(keys)}
            return all(abs(sc[pos[g]] - sc[order[j]]) <= 1e-2 for j, g in enumerate(got))
        s, ks = res[0]["scores"], res[0]["keys"]
        v["search_ok"] = bool(all(matches(q[b], flt[b], 4, s[b], ks[b]) for b in range(2)))
        es = res[1]
        v["embed_search_ok"] = bool(es["vecs"].shape == (1, eng.dim) and np.allclose(es["vecs"][0], allv[7], atol=1e-5)
                                    and matches(es["vecs"][0], docs, 3, es["scores"][0], es["keys"][0]))
        v["answers_ok"] = all(0.0 <= r["results"][0][1] <= 0.5 + 1e-6 for r in res[3:])
        await slow
        v["slow_done"] = True
        # load balancing: concurrent answers spread over the replicas
        await asyncio.gather(*[cl.call("answer", items=[{"question": f"lb{i}", "context": "c", "quality": 1.0}])
                               for i in range(2 * cl.replicas)])
        st = await cl.call("stats")
        v["answered_per_replica"] = [sum(r.get("gen", {}).get("calls", 0) + r.get("sched", {}).get("admitted", 0)
                                         for r in part["ranks"][:1]) for part in st["replicas"]]
        await cl.close()
        return v

    asyncio.run(serve())
    plane.stop()
    dist.barrier()
    dist.destroy_process_group()


def check_ivf_kmeans(rank, world, port, out_path):
    _init(rank, world, port)
    from docagents_amd.index.ivf import IVFFlatIndex
    from docagents_amd.parallel.sharded_index import ShardedIndex
    d, per = 32, 600
    rng = np.random.default_rng(1)
    centers = rng.standard_normal((8, d)).astype(np.float32)
    lab = rng.integers(0, 8, size=world * per)
    X = centers[lab] + 0.15 * rng.standard_normal((world * per, d)).astype(np.float32)
    X /= np.linalg.norm(X, axis=1, keepdims=True)
    ix = IVFFlatIndex(d, "cpu", lists=8, probes=2)
    lo = rank * per
    for r0 in range(lo, lo + per, 50):
        ix.add(f"d{r0}", np.arange(r0, r0 + 50), torch.from_numpy(X[r0:r0 + 50]))
    sh = ShardedIndex(ix, rank, world)
    sh.train(iters=8)
    Q = X[rng.choice(world * per, 20, replace=False)] + 0.01
    Q /= np.linalg.norm(Q, axis=1, keepdims=True)
    s, ids = sh.search(torch.from_numpy(Q[rank * 10:(rank + 1) * 10] if rank < 2 else Q[:10]), 5, -1.0, None)
    # recall@5 vs exact
    rec = []
    for b in range(ids.shape[0]):
        qi = rank * 10 + b if rank < 2 else b
        exact = set(np.argsort(-(X @ Q[qi]))[:5].tolist())
        rec.append(len(exact & set(ids[b].tolist())) / 5)
    allrec = [None] * world
    dist.all_gather_object(allrec, float(np.mean(rec)))
    C = ix.centroids.float()
    C0 = C.clone()
    dist.broadcast(C0, 0)
    _done(rank, out_path, {"recall": float(np.mean(allrec)), "centroids_equal": bool(torch.allclose(C, C0))})


def check_xgmi_allreduce(rank, world, port, out_path):
    """XgmiAllReduce (IPC peer buffers, ops/csrc/allreduce.hip) == the fp32 rank-order sum, for
    one-shot and two-shot sizes, bf16 and fp32, eager and HIP-graph replay, with back-to-back calls
    of different sizes (exercises the per-workgroup counters and the staging parity). GPU ranks;
    the handle exchange rides a gloo group, so several ranks may share one GPU (1-GPU rehearsal)."""
    _init(rank, world, port)
    from docagents_amd.parallel.xgmi_allreduce import XgmiAllReduce
    dev = torch.device("cuda", rank % torch.cuda.device_count())
    torch.cuda.set_device(dev)
    ar = XgmiAllReduce(None, dev, max_bytes=8 << 20, oneshot_max=256 << 10)
    verdict = {"cases": [], "ok": True}

    def inputs(n, dtype, salt):
        xs = []
        for r in range(world):
            g = torch.Generator(device="cpu").manual_seed(1000 * salt + r)
            xs.append(torch.randn(n, generator=g).to(dtype))
        return xs

    def ref_sum(xs, dtype):
        acc = torch.zeros_like(xs[0], dtype=torch.float32)
        for x in xs:
            acc += x.float()
        return acc.to(dtype)

    sizes = [8, 4096, 8192 * 3, 131072, 8192 * 64, 1_000_000, (8 << 20) // 2]
    salt = 0
    for dtype in (torch.bfloat16, torch.float32):
        for n in sizes:
            if n * (2 if dtype == torch.bfloat16 else 4) > (8 << 20):
                continue
            salt += 1
            xs = inputs(n, dtype, salt)
            t = xs[rank].to(dev)
            ar.all_reduce_(t)
            torch.cuda.synchronize()
            ref = ref_sum(xs, dtype)
            err = float((t.cpu().float() - ref.float()).abs().max())
            ok = err == 0.0
            verdict["cases"].append({"n": n, "dtype": str(dtype), "max_err": err, "ok": ok})
            verdict["ok"] &= ok
    # graph capture: three calls (one-shot, two-shot, one-shot) replayed twice with fresh inputs
    bufs = [torch.empty(n, dtype=torch.bfloat16, device=dev) for n in (8192, 400_000, 16384)]
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for b in bufs:  # warm-up outside capture
            b.zero_()
            ar.all_reduce_(b)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        for b in bufs:
            ar.all_reduce_(b)
    for rep in range(2):
        refs = []
        for i, b in enumerate(bufs):
            salt += 1
            xs = inputs(b.numel(), torch.bfloat16, salt)
            b.copy_(xs[rank].to(dev))
            refs.append(ref_sum(xs, torch.bfloat16))
        graph.replay()
        torch.cuda.synchronize()
        for b, ref in zip(bufs, refs):
            err = float((b.cpu().float() - ref.float()).abs().max())
            verdict["cases"].append({"n": b.numel(), "graph_replay": rep, "max_err": err, "ok": err == 0.0})
            verdict["ok"] &= err == 0.0
    ar.check()
    verdict["calls"] = ar.calls
    ar.close()
    _done(rank, out_path, verdict)


def check_xgmi_verify_and_time(rank, world, port, out_path):
    """The cross-device check bench.py runs on multi-GPU nodes (xgmi_allreduce.verify_and_time),
    rehearsed with ranks that may share one GPU."""
    _init(rank, world, port)
    from docagents_amd.parallel.xgmi_allreduce import verify_and_time
    dev = torch.device("cuda", rank % torch.cuda.device_count())
    torch.cuda.set_device(dev)
    _done(rank, out_path, verify_and_time(None, dev, iters=10))


def check_xgmi_reuse(rank, world, port, out_path):
    """Communicators created, used and closed repeatedly in one process, as bench.py's N > 1 blocks
    do (TP model + its norm communicator, closed; the verdict's pair, closed; a third size): every
    all-reduce exact, the pooled buffers reused for a size seen before."""
    _init(rank, world, port)
    import docagents_amd.parallel.xgmi_allreduce as X
    dev = torch.device("cuda", rank % torch.cuda.device_count())
    torch.cuda.set_device(dev)
    verdict = {"rounds": [], "ok": True}
    for rnd, sizes in enumerate([(32 << 20, 512 << 10), (32 << 20, 512 << 10), (16 << 20,), (32 << 20,)]):
        comms = [X.XgmiAllReduce(None, dev, max_bytes=b) for b in sizes]
        for i, c in enumerate(comms):
            n = 64 * 3072 + 8 * i
            x = torch.full((n,), float(rank + 1 + rnd), dtype=torch.float32, device=dev)
            c.all_reduce_(x)
            torch.cuda.synchronize(dev)
            want = sum(r + 1 + rnd for r in range(world))
            ok = bool((x == want).all())
            verdict["rounds"].append({"round": rnd, "max_bytes": sizes[i], "ok": ok})
            verdict["ok"] &= ok
        dist.barrier()
        for c in comms:
            c.close()
    verdict["pooled_sizes"] = sorted(k[1] for k in X._POOL)
    verdict["pooled_buffers"] = sum(len(v) for v in X._POOL.values())
    _done(rank, out_path, verdict)


def check_xgmi_allreduce_norm(rank, world, port, out_path):
    """C3 with the RMSNorm in the all-reduce's epilogue (one launch) vs the all-reduce kernel
    followed by the rmsnorm kernel: x and h must be BIT-identical, for several row widths / row
    counts, gamma given or unit, eager and HIP-graph replay. GPU ranks (may share one GPU)."""
    _init(rank, world, port)
    from docagents_amd.ops import kernels as K
    from docagents_amd.parallel.xgmi_allreduce import XgmiAllReduce
    dev = torch.device("cuda", rank % torch.cuda.device_count())
    torch.cuda.set_device(dev)
    plain = XgmiAllReduce(None, dev, max_bytes=8 << 20)
    verdict = {"cases": [], "ok": True}
    salt = 0
    for D in (256, 3072, 8192):
        fused = XgmiAllReduce(None, dev, max_bytes=512 << 10)  # one row width per instance
        for rows in (1, 4, 31):
            if rows * D * 2 > (512 << 10):
                continue
            for with_gamma in (False, True):
                salt += 1
                g = torch.Generator().manual_seed(salt)
                xs = [torch.randn(rows, D, generator=g).bfloat16() for _ in range(world)]
                gamma = (torch.rand(D, generator=g) + 0.5).bfloat16().to(dev) if with_gamma else None
                x1 = xs[rank].to(dev)
                h1 = torch.empty_like(x1)
                fused.all_reduce_rmsnorm_(x1, gamma, 1e-5, h1)
                x2 = xs[rank].to(dev)
                plain.all_reduce_(x2)
                h2 = K.rmsnorm(x2, gamma if gamma is not None else torch.ones(D, dtype=torch.bfloat16, device=dev),
                               1e-5)
                torch.cuda.synchronize()
                ok = bool(torch.equal(x1, x2) and torch.equal(h1, h2))
                verdict["cases"].append({"D": D, "rows": rows, "gamma": with_gamma, "ok": ok,
                                         "max_h_err": float((h1.float() - h2.float()).abs().max())})
                verdict["ok"] &= ok
        if D == 3072:  # graph capture of two fused calls, replayed with fresh inputs
            x = torch.zeros(4, D, dtype=torch.bfloat16, device=dev)
            h = torch.empty_like(x)
            s_ = torch.cuda.Stream()
            s_.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s_):
                fused.all_reduce_rmsnorm_(x, None, 1e-5, h)
            torch.cuda.current_stream().wait_stream(s_)
            torch.cuda.synchronize()
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph):
                fused.all_reduce_rmsnorm_(x, None, 1e-5, h)
                fused.all_reduce_rmsnorm_(x, None, 1e-5, h)
            for rep in range(2):
                salt += 1
                g = torch.Generator().manual_seed(salt)
                xs = [torch.randn(4, D, generator=g).bfloat16() for _ in range(world)]
                x.copy_(xs[rank].to(dev))
                graph.replay()
                torch.cuda.synchronize()
                acc = torch.zeros(4, D)
                for xx in xs:
                    acc += xx.float()
                once = acc.bfloat16()  # first call: the sum; second: world x the sum
                acc2 = torch.zeros(4, D)
                for _ in range(world):
                    acc2 += once.float()
                want = acc2.bfloat16().to(dev)
                hw = K.rmsnorm(want, torch.ones(D, dtype=torch.bfloat16, device=dev), 1e-5)
                ok = bool(torch.equal(x, want) and torch.equal(h, hw))
                verdict["cases"].append({"D": D, "graph_replay": rep, "ok": ok})
                verdict["ok"] &= ok
        fused.check()
        fused.close()
    plain.check()
    plain.close()
    _done(rank, out_path, verdict)


def check_tp_decoder_gpu(rank, world, port, out_path, wrong_order: bool = False):
    """TP=world LlamaDecoder on GPU ranks (row-parallel outputs summed by the xGMI all-reduce kernel,
    vocab-parallel sampling gathered over it) vs the unsharded decoder on the same device, with the
    per-decision verdict of check_tp_decoder. ``wrong_order``: negative control."""
    _init(rank, world, port)
    from docagents_amd.parallel.tp_verify import decision_verdict
    dev = torch.device("cuda", rank % torch.cuda.device_count())
    torch.cuda.set_device(dev)
    _done(rank, out_path, decision_verdict(rank, world, None, dev, wrong_order=wrong_order))


def check_tp_decoder_gpu_wrong_order(rank, world, port, out_path):
    check_tp_decoder_gpu(rank, world, port, out_path, wrong_order=True)


def check_replica_failover(rank, world, port, out_path, victim: int | None = None):
    """Replicas fail independently (the reference's queue-group workers, internal/queue/nats.go:40-51,
    docker-compose.yml:84-85): ``world`` one-rank replicas serve the full stack as engine_main builds
    it; once ingest is done the ``victim`` rank (default: the last) SIGKILLs itself. Then, driven by
    rank 0 through ``EngineCluster``: searches over documents on live ranks must keep returning the
    exact result, searches that need the dead shard must fail (naming it), answers must keep flowing
    (retried away from the dead replica), and ``health`` must name the dead replica and shard.
    Coordination after the kill uses files only: no collective can run with a dead member."""
    import asyncio
    import signal
    import time as _t
    _init(rank, world, port)
    from docagents_amd.engine.engine import Engine
    from docagents_amd.engine.rpc import EngineCluster
    from docagents_amd.engine.server import EngineGroup, EngineServer, owner_of
    from docagents_amd.utils.log import discard
    from docagents_amd.parallel.search_plane import SearchPlane
    victim = world - 1 if victim is None else victim
    eng = Engine("tiny-enc", "tiny-dec", "cpu", max_batch=4, max_seq=512, max_new_tokens=4, summary_max_new=4,
                 use_graphs=False)
    plane = SearchPlane.start_world(eng.index, rank, world, None, timeout_s=10.0, retry_s=0.2)
    grp = EngineGroup(eng, rank, world, plane=plane)
    ports = [0] * world
    if rank == 0:
        socks = [socket.socket() for _ in range(world)]
        for sk in socks:
            sk.bind(("127.0.0.1", 0))
        ports = [sk.getsockname()[1] for sk in socks]
        for sk in socks:
            sk.close()
    box = [ports]
    dist.broadcast_object_list(box, src=0)
    urls = [f"tcp://127.0.0.1:{p}" for p in box[0]]
    kill_flag, done_flag = out_path + ".kill", out_path + ".done"

    async def serve():
        srv = EngineServer(grp, discard(), continuous=True, cb_window_s=0.0, urls=urls, liveness_s=0)
        await srv.start(urls[rank])
        if rank == 0:
            try:
                verdict = await drive()
            except Exception as e:  # noqa: BLE001 - reported, the test asserts on it
                verdict = {"error": repr(e)}
            with open(out_path, "w") as f:
                json.dump(verdict, f)
            open(done_flag, "w").close()
        else:
            while not os.path.exists(done_flag):
                if rank == victim and os.path.exists(kill_flag):
                    os.kill(os.getpid(), signal.SIGKILL)
                await asyncio.sleep(0.02)
        srv.server.close()

    async def drive():
        v = {}
        cl = await EngineCluster(urls[0], timeout=30.0).connect(retries=200, delay=0.05)
        docs, per = [], {}
        i = 0
        while min(per.get(r, 0) for r in range(world)) < 2:
            d = f"fo-doc-{i}"
            i += 1
            o = owner_of(d, world)
            if per.get(o, 0) < 2:
                docs.append(d)
                per[o] = per.get(o, 0) + 1
        texts = {d: [f"chunk {j} of {d} on topic {i * 5 + j}" for j in range(3)] for i, d in enumerate(docs)}
        await asyncio.gather(*[cl.call("embed_index", doc_id=d, keys=np.arange(3, dtype=np.int64) + 10 * i,
                                       texts=texts[d]) for i, d in enumerate(docs)])
        allt = [t for d in docs for t in texts[d]]
        allv = (await cl.clients[0].call("embed", texts=allt, preprocess=True))["vecs"]
        keys = np.array([10 * i + j for i, _ in enumerate(docs) for j in range(3)])
        live = [d for d in docs if owner_of(d, world) != victim]
        dead_docs = [d for d in docs if owner_of(d, world) == victim]

        def exact(q, allowed, k):
            m = np.array([d in allowed for d in docs for _ in range(3)])
            sc = allv @ q
            idx = np.where(m)[0]
            order = idx[np.lexsort((idx, -sc[idx]))][:k]
            return sc[order], keys[order]

        def ok(res, q, allowed, k):
            s_ref, _ = exact(q, allowed, k)
            got = [x for x in res["keys"][0] if x >= 0]
            return len(got) == len(s_ref) and np.allclose(np.sort(res["scores"][0][:len(got)]), np.sort(s_ref),
                                                          atol=1e-2)
        q = allv[4]
        v["before_all_ok"] = ok(await cl.call("search", vecs=q[None], filters=[docs], k=5, min_sim=-1.0), q, docs, 5)
        open(kill_flag, "w").close()
        t0 = _t.perf_counter()
        while _t.perf_counter() - t0 < 30:
            h = await cl.call("health")
            if victim in h.get("dead_replicas", []):
                break
            await asyncio.sleep(0.1)
        v["dead_detected_s"] = round(_t.perf_counter() - t0, 3)
        # searches over live shards, issued at every live replica
        res = []
        for r in range(world):
            if r == victim:
                continue
            for b in range(3):
                qq = allv[(3 * b + r) % len(allv)]
                rr = await cl.clients[r].call("search", vecs=qq[None], filters=[live], k=4, min_sim=-1.0)
                res.append(ok(rr, qq, live, 4))
        v["live_searches_ok"] = bool(res) and all(res)
        try:
            await cl.clients[0].call("search", vecs=q[None], filters=[[live[0], dead_docs[0]]], k=4, min_sim=-1.0)
            v["dead_search_failed"] = False
        except Exception as e:  # noqa: BLE001
            v["dead_search_failed"] = f"shard {victim}" in str(e)
            v["dead_search_error"] = str(e)[:200]
        answers = await asyncio.gather(*[cl.call("answer", items=[{"question": f"q{i}?", "context": "ctx",
                                                                   "quality": 0.5}]) for i in range(2 * world)],
                                       return_exceptions=True)
        v["answers_ok"] = all(not isinstance(a, BaseException) and 0.0 <= a["results"][0][1] <= 0.5 + 1e-6
                              for a in answers)
        v["answer_errors"] = [repr(a)[:120] for a in answers if isinstance(a, BaseException)]
        es = await cl.call("embed_search", texts=[allt[1]], filters=[live], k=3, min_sim=-1.0)
        v["embed_search_ok"] = bool(ok(es, es["vecs"][0], live, 3))
        h = await cl.call("health")
        v["health_ok_flag"] = h["ok"]
        v["dead_replicas"] = h.get("dead_replicas")
        v["shards_down"] = h.get("shards_down")
        await cl.close()
        return v

    asyncio.run(serve())
    plane.stop(timeout=2.0)
    os._exit(0)  # no collective teardown: the process group has a dead member
